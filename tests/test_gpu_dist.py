"""GPU, world size 2: the N>1 path as bench.py runs it -- one process per
rank, each hashing its own contiguous slice of a global batch on its device
through the C ABI, no data-path collective -- and the gathered slices equal
the oracle's digests of the whole batch (bit-exact).

On the 1-GPU box both ranks share cuda:0 (device = rank mod device count,
as bench.py does) and talk over gloo; the 8-GPU runs are the driver's.
Fixed layout with equal-count shards, and the variable layout with
byte-balanced shards whose offsets are rebased per rank."""
import os
import socket

import numpy as np
import pytest

import synth
from ilias_net2_amd import shard

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N_FIXED, LEN_FIXED = 20011, 1024
N_VAR = 12007


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from ilias_net2_amd import batch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", rank % torch.cuda.device_count())
        torch.cuda.set_device(dev)
        # fixed layout: only this rank's packets travel to its device
        data = synth.fixed_batch(41, N_FIXED, LEN_FIXED)
        lo, hi = shard.shard_range(N_FIXED, world, rank)
        mine = torch.from_numpy(data[lo * LEN_FIXED:hi * LEN_FIXED]).to(dev)
        local = batch.digest_fixed(1, mine, LEN_FIXED, LEN_FIXED, hi - lo)
        full = shard.gather_digests(local.cpu().numpy())
        # variable layout, byte-balanced, SHA-512
        lens = synth.mixed_lengths(42, N_VAR)
        vdata, offs = synth.packed(43, lens)
        cuts = shard.shard_cuts_by_bytes(lens, world)
        a, b = cuts[rank], cuts[rank + 1]
        base = int(offs[a]) if b > a else 0
        end = int(offs[b - 1] + lens[b - 1]) if b > a else 0
        vmine = torch.from_numpy(vdata[base:end]).to(dev)
        voffs = torch.from_numpy((offs[a:b] - np.uint64(base)).astype(np.int64)).to(dev)
        vlens = torch.from_numpy(lens[a:b].astype(np.int32)).to(dev)
        vlocal = batch.digest_var(3, vmine, voffs, vlens)
        torch.cuda.synchronize(dev)
        vfull = shard.gather_digests(vlocal.cpu().numpy())
        if rank == 0:
            q.put((full, vfull))
    finally:
        dist.destroy_process_group()


def test_two_ranks_on_gpu(oracle_mod):
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a GPU (HIP device not visible)")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        full, vfull = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    data = synth.fixed_batch(41, N_FIXED, LEN_FIXED)
    want = oracle_mod.batch(1, data, stride=LEN_FIXED, length=LEN_FIXED,
                            n=N_FIXED, nthreads=8)
    assert np.array_equal(full, want)
    lens = synth.mixed_lengths(42, N_VAR)
    vdata, offs = synth.packed(43, lens)
    assert np.array_equal(vfull, oracle_mod.batch(3, vdata, offsets=offs,
                                                  lens=lens, nthreads=8))

"""CPU, world size 2 over gloo: the N>1 path shards a global batch into
contiguous per-rank slices with no data-path collective, and the slices'
digests reassemble into the single-process result.

The per-rank compute here is the CPU oracle (no GPU in this container); on
the GPU box the same slices go through net2_sha2_batch / dev_* per rank."""
import os
import socket

import numpy as np
import pytest

import synth
from ilias_net2_amd import shard


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_range_covers():
    for n in (0, 1, 7, 1000, 1 << 20):
        for w in (1, 2, 3, 8):
            parts = [shard.shard_range(n, w, r) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))


def test_shard_by_bytes_balanced():
    lens = synth.mixed_lengths(3, 100000)
    for w in (2, 4, 8):
        cuts = shard.shard_cuts_by_bytes(lens, w)
        assert cuts[0] == 0 and cuts[-1] == len(lens)
        assert cuts == sorted(cuts)
        per = [int(lens[a:b].sum()) for a, b in zip(cuts, cuts[1:])]
        assert max(per) - min(per) <= 2 * 1500 + 1, per


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from oracle import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # fixed layout, equal-count shards
        n, length = 3001, 200
        data = synth.fixed_batch(31, n, length)
        lo, hi = shard.shard_range(n, world, rank)
        local = oracle.batch(1, data[lo * length:hi * length], stride=length,
                             length=length, n=hi - lo)
        full = shard.gather_digests(local)
        # variable layout, byte-balanced shards
        lens = synth.mixed_lengths(32, 2500)
        vdata, offs = synth.packed(33, lens)
        cuts = shard.shard_cuts_by_bytes(lens, world)
        a, b = cuts[rank], cuts[rank + 1]
        vlocal = oracle.batch(3, vdata, offsets=offs[a:b], lens=lens[a:b])
        vfull = shard.gather_digests(vlocal)
        if rank == 0:
            q.put((full, vfull))
    finally:
        dist.destroy_process_group()


def test_two_ranks_gloo():
    import torch.multiprocessing as mp
    from oracle import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    full, vfull = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n, length = 3001, 200
    data = synth.fixed_batch(31, n, length)
    assert np.array_equal(full, oracle.batch(1, data, stride=length, length=length, n=n))
    lens = synth.mixed_lengths(32, 2500)
    vdata, offs = synth.packed(33, lens)
    assert np.array_equal(vfull, oracle.batch(3, vdata, offsets=offs, lens=lens))


# ---- the N>1 bench line --------------------------

def _bench_worker(rank, world, port, q, pcis):
    import torch.distributed as dist
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        gpu = {"host": "box-a", "pci": pcis[rank]}
        ranks = bench.gather_ranks(bench.rank_record(rank, gpu, 1.0 + rank), world)
        out = {"ranks": ranks, "gloo": bench.scale_fields(ranks, "gloo")}
        try:
            bench.scale_fields(ranks, "nccl")
            out["nccl"] = "accepted"
        except SystemExit as e:
            out["nccl"] = "refused: " + str(e)
        # cpu_baseline at N>1: rank 0 times the host after the GPU steps,
        # the other ranks wait on the store (no spinning, no deadlock)
        cb = bench.cpu_baseline_after_gpu({"n": 1}, rank, world,
                                          fn=lambda cfg: {"value": 42.0, "cores": 16})
        out["cpu_baseline"] = cb
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("shared", [True, False])
def test_bench_rank_records_gloo(shared):
    """Two gloo ranks build the N>1 line's device fields: every rank's PCI
    id, host, NUMA node and own ms_per_step; min / max over ranks; two ranks
    on one device are labelled "shared device" under gloo and refused under
    RCCL (the driver's backend); distinct devices pass both.  rank 0 alone
    carries cpu_baseline."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    pcis = ["0000:05:00.0", "0000:05:00.0"] if shared else ["0000:05:00.0", "0000:15:00.0"]
    procs = [ctx.Process(target=_bench_worker, args=(r, 2, port, q, pcis))
             for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in (0, 1):
        o = got[rank]
        assert [r["rank"] for r in o["ranks"]] == [0, 1]
        assert [r["pci"] for r in o["ranks"]] == pcis
        assert all(set(r) >= {"host", "numa_node", "ms_per_step"} for r in o["ranks"])
        g = o["gloo"]
        assert g["ms_per_step_ranks"] == {"min": 1.0, "max": 2.0}
        if shared:
            assert g["distinct_devices"] == 1
            assert g["device_sharing"].startswith("shared device")
            assert o["nccl"].startswith("refused")
        else:
            assert g["distinct_devices"] == 2
            assert g["device_sharing"] == "one GPU per rank"
            assert o["nccl"] == "accepted"
    assert got[0]["cpu_baseline"] == {"value": 42.0, "cores": 16}
    assert got[1]["cpu_baseline"] is None
    import bench
    assert bench.devices_label(2, 1) == "2 ranks on 1 shared GPU(s)"
    assert bench.devices_label(8, 8) == "8 GPU(s)"

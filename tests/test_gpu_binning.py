"""The one-pass length binning (bin_onepass_kernel):
one launch counts, scans and scatters, keeping its state in the caller's
workspace and cleaning up after itself.  Checked through the C ABI: every
digest against the oracle, and the visiting order itself (the perm words of
the workspace) -- a permutation of the batch, longest block count first
when binned, submission order when the workspace was not prepared or the
grid barrier was decided ABORT."""
import os
import subprocess
import sys

import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a GPU (HIP device not visible)")
    return torch.device("cuda:0")


def _hdr_words(L):
    return L.net2_sha2_dev_var_workspace(0) // 4


def _blocks(lens, alg):
    blk, lb = (64, 8) if alg == 1 else (128, 16)
    return (lens.astype(np.int64) + lb + 1 + blk - 1) // blk


def _order(ws, L, n):
    return ws.cpu().numpy()[_hdr_words(L):_hdr_words(L) + n].astype(np.int64)


@pytest.mark.parametrize("alg", [1, 3])
def test_workspace_lifecycle(dev, oracle_mod, alg):
    """An unprepared (zeroed) workspace: the first call hashes in submission
    order while it prepares itself; the next calls bin (block counts
    non-increasing along the order), the epoch advancing every call, the
    two parities alternating -- every digest right throughout."""
    from ilias_net2_amd import _lib, batch
    L = _lib.lib()
    n = 300_000
    lens = synth.mixed_lengths(600 + alg, n, choices=(0, 64, 200, 512, 1500, 3000))
    data, offs = synth.packed(610 + alg, lens, align=1)
    want = oracle_mod.batch(alg, data, offsets=offs, lens=lens, nthreads=16)
    d = torch.from_numpy(data).to(dev)
    o = torch.from_numpy(offs.astype(np.int64)).to(dev)
    ln = torch.from_numpy(lens.astype(np.int32)).to(dev)
    ws = torch.zeros(L.net2_sha2_dev_var_workspace(n) // 4, dtype=torch.int32,
                     device=dev)
    bl = _blocks(lens, alg)
    for call in range(6):
        got = batch.digest_var(alg, d, o, ln, workspace=ws)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy(), want), call
        order = _order(ws, L, n)
        assert np.array_equal(np.sort(order), np.arange(n)), call
        if call == 0:
            assert np.array_equal(order, np.arange(n))
        else:
            assert (np.diff(bl[order]) <= 0).all(), call
    # epoch counts the binned launches (header word 2); the barrier words
    # (after the header and the two parities of the 2,048-bin histogram,
    # 1,024 per parity: group counters every 32 words, top counter
    # at 512, state at 544) -- the last launch's parity (0) decided GO with
    # every workgroup arrived, the next one's zeroed
    w = ws.cpu().numpy().view(np.uint32)
    assert w[2] == 5, w[:8]
    ctl0 = 16 + 2 * 2048
    ctl = w[ctl0:ctl0 + 2 * 1024].reshape(2, 1024)
    G = min(256, (n + 4095) // 4096)
    assert ctl[0, 544] == 1 and ctl[0, 512] == min(G, 16), ctl[0, [512, 544]]
    assert ctl[0, 0:512:32].sum() == G
    assert not ctl[1, 0:512:32].any() and ctl[1, 512] == 0 and ctl[1, 544] == 0


def test_prepared_workspace_bins_from_the_first_call(dev, oracle_mod):
    from ilias_net2_amd import _lib, batch
    L = _lib.lib()
    n = 100_000
    lens = synth.mixed_lengths(620, n)
    data, offs = synth.packed(621, lens)
    ws = batch.var_workspace(n, dev)      # net2_sha2_workspace_init
    got = batch.digest_var(1, torch.from_numpy(data).to(dev),
                           torch.from_numpy(offs.astype(np.int64)).to(dev),
                           torch.from_numpy(lens.astype(np.int32)).to(dev),
                           workspace=ws)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(),
                          oracle_mod.batch(1, data, offsets=offs, lens=lens))
    order = _order(ws, L, n)
    assert (np.diff(_blocks(lens, 1)[order]) <= 0).all()
    assert L.net2_sha2_workspace_init(None, 0, None) == 22


@pytest.mark.parametrize("n", [1, 4096, 4097, 15 * 4096 + 7, 16 * 4096,
                               17 * 4096 + 1, 33 * 4096 + 5])
def test_grid_sizes_around_the_barrier_groups(dev, oracle_mod, n):
    """G = 1 .. 34 workgroups: groups of one, groups of two, a partial
    top level (G < 16) -- each launch decides GO with every workgroup
    counted once, two launches in a row (both parities)."""
    from ilias_net2_amd import _lib, batch
    L = _lib.lib()
    lens = synth.mixed_lengths(650 + n % 97, n, choices=(0, 64, 300, 1500))
    data, offs = synth.packed(651, lens)
    if data.size == 0:
        data = np.zeros(1, dtype=np.uint8)
    want = oracle_mod.batch(3, data, offsets=offs, lens=lens, nthreads=16)
    d = torch.from_numpy(data).to(dev)
    o = torch.from_numpy(offs.astype(np.int64)).to(dev)
    ln = torch.from_numpy(lens.astype(np.int32)).to(dev)
    ws = batch.var_workspace(n, dev)
    G = min(256, (n + 4095) // 4096)
    for call in range(2):
        got = batch.digest_var(3, d, o, ln, workspace=ws)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy(), want), (n, call)
        order = _order(ws, L, n)
        assert np.array_equal(np.sort(order), np.arange(n))
        assert (np.diff(_blocks(lens, 3)[order]) <= 0).all()
        w = ws.cpu().numpy().view(np.uint32)
        assert w[2] == call + 1
        ctl = w[16 + 2 * 2048:16 + 2 * 2048 + 2 * 1024].reshape(2, 1024)[call & 1]
        assert ctl[544] == 1 and ctl[512] == min(G, 16), (n, call, ctl[[512, 544]])
        assert ctl[0:512:32].sum() == G


def test_many_tiles_per_workgroup(dev, oracle_mod):
    """3 M packets: 733 tiles over the 256-workgroup persistent grid (each
    workgroup bins three tiles), lengths over seven bins."""
    from ilias_net2_amd import _lib, batch
    L = _lib.lib()
    n = 3_000_000
    lens = synth.mixed_lengths(630, n, choices=(0, 1, 55, 56, 119, 200, 300))
    data, offs = synth.packed(631, lens)
    ws = batch.var_workspace(n, dev)
    got = batch.digest_var(3, torch.from_numpy(data).to(dev),
                           torch.from_numpy(offs.astype(np.int64)).to(dev),
                           torch.from_numpy(lens.astype(np.int32)).to(dev),
                           workspace=ws)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(),
                          oracle_mod.batch(3, data, offsets=offs, lens=lens,
                                           nthreads=16))
    order = _order(ws, L, n)
    assert np.array_equal(np.sort(order), np.arange(n))
    assert (np.diff(_blocks(lens, 3)[order]) <= 0).all()


_ABORT = r'''
import sys
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np, torch
import synth
from oracle import oracle
from ilias_net2_amd import batch, _lib
L = _lib.lib()
dev = torch.device("cuda:0")
n = 200_000
lens = synth.mixed_lengths(640, n)
data, offs = synth.packed(641, lens)
want = oracle.batch(1, data, offsets=offs, lens=lens, nthreads=16)
d = torch.from_numpy(data).to(dev)
o = torch.from_numpy(offs.astype(np.int64)).to(dev)
ln = torch.from_numpy(lens.astype(np.int32)).to(dev)
ws = batch.var_workspace(n, dev)
bad = 0
for _ in range(12):
    got = batch.digest_var(1, d, o, ln, workspace=ws)
    torch.cuda.synchronize()
    bad += not np.array_equal(got.cpu().numpy(), want)
    order = ws.cpu().numpy()[L.net2_sha2_dev_var_workspace(0) // 4:][:n]
    bad += not np.array_equal(np.sort(order), np.arange(n))
hm = batch.hmac_dev(6, bytes(64), d, offsets=o, lens=ln, workspace=ws)
torch.cuda.synchronize()
bad += not np.array_equal(hm.cpu().numpy()[::997], np.stack([
    np.frombuffer(oracle.hmac(6, bytes(64), data[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes()),
                  dtype=np.uint8) for i in range(0, n, 997)]))
print("BAD", bad)
'''


def test_barrier_timeout_takes_submission_order():
    """NET2_BIN_TIMEOUT_US=0: the grid barrier may be decided ABORT before
    every workgroup arrives -- then all of them take the submission order
    and the header re-initialises at the next call.  Whatever each call
    decides, its digests and order are right (fresh process)."""
    env = dict(os.environ, NET2_BIN_TIMEOUT_US="0")
    r = subprocess.run([sys.executable, "-c", _ABORT], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "BAD 0" in r.stdout, r.stdout + r.stderr

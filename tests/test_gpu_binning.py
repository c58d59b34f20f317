"""The one-pass length binning (bin_onepass_kernel): one launch counts, scans
and scatters, keeping its state in the caller's workspace and cleaning up
after itself.  Checked through the C ABI: every digest against the oracle,
the visiting order itself (the perm words of the workspace) -- a permutation
of the batch, longest block count first when binned, submission order when
the workspace was not prepared or the grid barrier was decided ABORT -- and
the workspace's counters (net2_sha2_workspace_stats): a fallback to
submission order is never silent."""
import os

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


def _stats(L, ws):
    from ilias_net2_amd import _lib
    torch.cuda.synchronize()
    return _lib.workspace_stats(ws.data_ptr(), ws.numel() * ws.element_size())


@pytest.fixture
def bin_limits():
    """net2_sha2_bin_limits for one test, the defaults restored after."""
    from ilias_net2_amd import _lib
    L = _lib.lib()
    yield lambda cap, timeout_us: L.net2_sha2_bin_limits(cap, timeout_us)
    L.net2_sha2_bin_limits(0, -1)


def _c3(n, seed, alg=1):
    lens = synth.mixed_lengths(seed, n)
    data, offs = synth.packed(seed + 1, lens)
    return lens, data, offs


def _dev_args(dev, data, offs, lens):
    return (torch.from_numpy(data).to(dev),
            torch.from_numpy(offs.astype(np.int64)).to(dev),
            torch.from_numpy(lens.astype(np.int32)).to(dev))


def test_barrier_timeout_takes_submission_order(dev, oracle_mod, bin_limits):
    """A zero barrier timeout: a launch whose workgroups are not all there
    when the first one polls is decided ABORT -- all of them take the
    submission order and the header re-initialises at the next call.
    Whatever each call decides, its digests and order are right, and every
    launch is accounted for: unprepared + aborted + binned."""
    from ilias_net2_amd import _lib, batch
    L = _lib.lib()
    bin_limits(0, 0)
    n = 200_000
    lens, data, offs = _c3(n, 640)
    want = oracle_mod.batch(1, data, offsets=offs, lens=lens, nthreads=16)
    d, o, ln = _dev_args(dev, data, offs, lens)
    ws = batch.var_workspace(n, dev)
    calls = 12
    for _ in range(calls):
        got = batch.digest_var(1, d, o, ln, workspace=ws)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy(), want)
        assert np.array_equal(np.sort(_order(ws, L, n)), np.arange(n))
    hm = batch.hmac_dev(6, bytes(64), d, offsets=o, lens=ln, workspace=ws)
    torch.cuda.synchronize()
    idx = range(0, n, 997)
    assert np.array_equal(hm.cpu().numpy()[::997], np.stack([
        np.frombuffer(oracle_mod.hmac(6, bytes(64), data[int(offs[i]):int(offs[i]) +
                      int(lens[i])].tobytes()), dtype=np.uint8) for i in idx]))
    st = _stats(L, ws)
    assert st["mismatches"] == 0
    assert st["unprepared"] + st["aborts"] + st["binned"] == calls + 1, st
    assert st["aborts"] > 0, st


def test_fresh_workspace_does_not_abort(dev, oracle_mod):
    """A fresh (zeroed) workspace under a full 256-workgroup grid: the first
    launch takes the submission order while workgroup 0 prepares the header;
    a workgroup dispatched after that must not mistake the header for a
    prepared one (it carries this launch's id) and join a barrier the early
    workgroups skipped -- no 50 ms stall, no abort.  The next launches bin."""
    from ilias_net2_amd import _lib, batch
    L = _lib.lib()
    n = 1 << 20
    lens, data, offs = _c3(n, 660)
    want = oracle_mod.batch(1, data, offsets=offs, lens=lens, nthreads=16)
    d, o, ln = _dev_args(dev, data, offs, lens)
    for rep in range(3):
        ws = torch.zeros(L.net2_sha2_dev_var_workspace(n) // 4, dtype=torch.int32,
                         device=dev)
        for call in range(3):
            got = batch.digest_var(1, d, o, ln, workspace=ws)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy(), want), (rep, call)
        st = _stats(L, ws)
        assert st == {"prepared": 1, "binned": 2, "aborts": 0, "mismatches": 0,
                      "unprepared": 1}, (rep, st)
        assert (np.diff(_blocks(lens, 1)[_order(ws, L, n)]) <= 0).all()


@pytest.mark.parametrize("cap", [1, 3, 40])
def test_grid_capped_below_the_tiles(dev, oracle_mod, bin_limits, cap):
    """The persistent grid capped (as on a partitioned device, or by
    net2_sha2_bin_limits): each workgroup bins many tiles, the barrier still
    completes, the order is binned."""
    from ilias_net2_amd import _lib, batch
    L = _lib.lib()
    bin_limits(cap, -1)
    n = 300_000
    lens, data, offs = _c3(n, 670)
    want = oracle_mod.batch(3, data, offsets=offs, lens=lens, nthreads=16)
    d, o, ln = _dev_args(dev, data, offs, lens)
    ws = batch.var_workspace(n, dev)
    for _ in range(2):
        got = batch.digest_var(3, d, o, ln, workspace=ws)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy(), want)
        order = _order(ws, L, n)
        assert np.array_equal(np.sort(order), np.arange(n))
        assert (np.diff(_blocks(lens, 3)[order]) <= 0).all()
    st = _stats(L, ws)
    assert st["binned"] == 2 and st["aborts"] == 0 and st["mismatches"] == 0, st


@pytest.mark.parametrize("nstreams", [2, 4])
def test_concurrent_streams_bin_without_aborts(dev, oracle_mod, nstreams):
    """C3 batches on several streams at once, each with its own workspace
    (DESIGN 5.6's two-stream overlap, and four): the binning grids run next
    to each other's hash kernels; every launch must still bin -- no barrier
    abort, block counts non-increasing along each order -- and every digest
    be right."""
    from ilias_net2_amd import _lib, batch
    L = _lib.lib()
    n = (1 << 20) // nstreams
    jobs = []
    for k in range(nstreams):
        lens, data, offs = _c3(n, 700 + k)
        want = oracle_mod.batch(1, data, offsets=offs, lens=lens, nthreads=16)
        d, o, ln = _dev_args(dev, data, offs, lens)
        jobs.append(dict(lens=lens, want=want, d=d, o=o, ln=ln,
                         ws=batch.var_workspace(n, dev),
                         out=torch.empty((n, 32), dtype=torch.uint8, device=dev),
                         s=torch.cuda.Stream(dev)))
    torch.cuda.synchronize()
    rounds = 8
    for _ in range(rounds):
        for j in jobs:
            with torch.cuda.stream(j["s"]):
                batch.digest_var(1, j["d"], j["o"], j["ln"], out=j["out"],
                                 workspace=j["ws"], stream=j["s"])
    torch.cuda.synchronize()
    for j in jobs:
        assert np.array_equal(j["out"].cpu().numpy(), j["want"])
        order = _order(j["ws"], L, n)
        assert np.array_equal(np.sort(order), np.arange(n))
        assert (np.diff(_blocks(j["lens"], 1)[order]) <= 0).all()
        st = _stats(L, j["ws"])
        assert st == {"prepared": 1, "binned": rounds, "aborts": 0,
                      "mismatches": 0, "unprepared": 0}, st


def test_overwritten_workspace_is_detected(dev, oracle_mod):
    """A caller reuses the workspace for other data between calls (here:
    stale counts in the next launch's histogram, then barrier counters that
    fire the grid barrier early): the binning finds that its histogram does
    not add up to the batch and the hash kernel falls back to submission
    order -- digests right, the mismatch counted, binning back two calls
    later."""
    from ilias_net2_amd import _lib, batch
    L = _lib.lib()
    n = 400_000
    lens, data, offs = _c3(n, 680)
    want = oracle_mod.batch(1, data, offsets=offs, lens=lens, nthreads=16)
    d, o, ln = _dev_args(dev, data, offs, lens)
    ws = batch.var_workspace(n, dev)
    hdr, nb = 16, 2048
    ctl0 = hdr + 2 * nb
    G = (n + 4095) // 4096

    def run():
        got = batch.digest_var(1, d, o, ln, workspace=ws)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy(), want)

    def epoch():
        torch.cuda.synchronize()
        return int(ws[2].item())

    run()
    assert epoch() == 1 and _stats(L, ws)["binned"] == 1
    par = epoch() & 1
    # 1. stale counts in the next parity's histogram
    ws[hdr + par * nb + 7] += 5
    run()
    st = _stats(L, ws)
    assert st["mismatches"] == 1 and not st["prepared"], st
    run()                                   # re-initialises: submission order
    run()                                   # binned again
    st = _stats(L, ws)
    assert st["prepared"] and st["unprepared"] == 1 and st["binned"] == 3, st
    assert (np.diff(_blocks(lens, 1)[_order(ws, L, n)]) <= 0).all()
    # 2. barrier words that decide GO at the first arrival: whatever the
    # workgroups then read, the digests stay right.  (The early decision also
    # bumps the epoch early: a workgroup that starts only after it reads the
    # next parity, joins that parity's barrier alone and waits out the
    # timeout -- an ABORT, counted, its counts a mismatch of the launch after.
    # Rare -- tools/forge_probe.py: none in 40 forged launches -- and only
    # with forged words: an honest barrier decides after every workgroup has
    # read the epoch.)
    for _ in range(3):
        base = ctl0 + (epoch() & 1) * 1024
        ws[base + 512] = min(G, 16) - 1     # top counter: one arrival short
        ws[base + 0] = (G + 15) // 16 - 1   # group 0: its first arrival is last
        run()
        run()
    st = _stats(L, ws)
    assert st["aborts"] <= 3, st
    # 3. the caller stops overwriting: every launch bins again, no fallback
    for _ in range(3):
        run()
    after = _stats(L, ws)
    run()
    run()
    final = _stats(L, ws)
    assert final["binned"] == after["binned"] + 2, (after, final)
    assert (final["aborts"], final["mismatches"]) == (after["aborts"],
                                                    after["mismatches"]), final
    assert (np.diff(_blocks(lens, 1)[_order(ws, L, n)]) <= 0).all()


def test_burst_workspace_reused_across_sizes(dev, oracle_mod):
    """One packet-burst workspace sized for the largest burst serves bursts
    of other sizes in turn (its binning area sits at offset 0 whatever n is,
    so another burst's status and verdict bytes can no longer land on the
    histogram); each burst mixes sealed and forged datagrams, every code
    against the oracle."""
    from ilias_net2_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(90)
    nmax, alg, ivlen = 200_000, 6, 16
    key = bytes(range(64))
    ws = torch.empty(L.net2_packet_burst_workspace(nmax), dtype=torch.uint8,
                     device=dev)
    st = torch.cuda.current_stream().cuda_stream
    for m in (nmax, 70_001, 150_000, 4096, nmax, 333, 199_999):
        lens = rng.choice(np.array([136, 584, 1500], dtype=np.uint32), m)
        offs = np.zeros(m, dtype=np.uint64)
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        data = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
        seq = rng.integers(0, 2**32, m, dtype=np.uint64).astype(np.uint32)
        flags = np.full(m, 3, dtype=np.uint32)
        r, sealed = oracle_mod.packet_encode_batch(alg, key, True, seq, flags, data,
                                                   offs, lens, nthreads=16)
        forged = rng.random(m) < 0.2       # sealed with the wrong key
        r2, sealed2 = oracle_mod.packet_encode_batch(alg, bytes(64), True, seq, flags,
                                                     data, offs, lens, nthreads=16)
        for i in np.nonzero(forged)[0]:
            a = int(offs[i])
            sealed[a:a + 72] = sealed2[a:a + 72]
        want = oracle_mod.packet_decode_batch(alg, key, True, ivlen, sealed, offs,
                                              lens, nthreads=16)
        assert np.array_equal(want[0] != 0, forged)
        d = torch.from_numpy(sealed).to(dev)
        o = torch.from_numpy(offs.view(np.int64)).to(dev)
        ln = torch.from_numpy(lens.view(np.int32)).to(dev)
        res = torch.full((m,), 9, dtype=torch.uint8, device=dev)
        iv = torch.zeros((m, ivlen), dtype=torch.uint8, device=dev)
        assert L.net2_packet_decode_burst(alg, key, 64, 1, ivlen, d.data_ptr(),
                                          o.data_ptr(), ln.data_ptr(), m,
                                          res.data_ptr(), iv.data_ptr(), None, None,
                                          ws.data_ptr(), ws.numel(), st) == 0
        assert np.array_equal(res.cpu().numpy(), want[0]), m
        ok = want[0] == 0
        assert np.array_equal(iv.cpu().numpy()[ok], want[1][ok]), m
    s = _lib.workspace_stats(ws.data_ptr(), ws.numel())
    assert s["aborts"] == 0 and s["mismatches"] == 0, s

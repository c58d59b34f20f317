"""bench.py's roofline join on the CPU: which committed counters reach a line
(the kernel build and the shader clock must match the line's), and the issue
floor of the dominant kernel and of the whole step."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

BUILD = "0123456789abcdef"
MIX = {"mean_issue_cycles_per_valu_instr": 3.951}


def _pmc(clock_ghz=2.39, build=BUILD, step=True):
    p = {"kernel_build_id": build, "clock_ghz_under_pmc": clock_ghz,
         "hbm_bytes_per_launch": 1.5e9, "valu_wave_instr_per_launch": 385.2e6,
         "trace_box": {"pci": "0000:00:00.0", "sclk_mhz_during_timed_steps": 2380}}
    if step:
        # the burst RX step: binning, the HMAC kernel, the final (IV) kernel
        p["step_kernels_valu"] = {
            "bin_onepass_kernel": {"dispatches": 500, "median_per_dispatch": 0.7e6},
            "hmac_kernel<Sha512H, false, 3, false>": {"dispatches": 500,
                                                      "median_per_dispatch": 385.2e6},
            "burst_final_kernel": {"dispatches": 500, "median_per_dispatch": 23.7e6}}
        p["step_valu_wave_instr"] = 0.7e6 + 385.2e6 + 23.7e6
    return p


@pytest.fixture
def joined(monkeypatch):
    """rooflines() with a stand-in counters file and ISA mix for one call."""
    def run(pmc, fresh=True, mix=MIX, launch_ms=0.7155, sclk=2380):
        monkeypatch.setattr(bench, "load_pmc", lambda name: (pmc, fresh))
        monkeypatch.setattr(bench, "load_isa_mix", lambda name: mix)
        monkeypatch.setattr(bench, "library_build_id", lambda: BUILD)
        return bench.rooflines("burst_rx", launch_ms, 815_000_000, sclk_mhz=sclk)
    return run


def test_counters_of_this_build_and_clock_are_joined(joined):
    roof, valu = joined(_pmc())
    assert roof["traffic"] == 1.5e9 and roof["traffic_build_id"] == BUILD
    assert roof["traffic_over_algorithmic"] == round(1.5e9 / 815e6, 3)
    assert roof["counters_clock_mhz"] == 2390
    floor = valu["issue_floor"]
    # dominant kernel: 385.2 M instructions x 3.951 cycles / 1024 SIMDs at
    # the line's 2,380 MHz against the 0.7155 ms of every launch of the step
    want = 385.2e6 / 1024 * 3.951 / 2380e6 * 1e3
    assert floor["floor_ms_at_timed_sclk"] == pytest.approx(want, abs=1e-4)
    assert floor["frac_at_timed_sclk"] == pytest.approx(want / 0.7155, abs=1e-4)
    # the whole step: every launch's VALU work priced the same way
    step = floor["step"]
    want_s = (0.7e6 + 385.2e6 + 23.7e6) / 1024 * 3.951 / 2380e6 * 1e3
    assert step["floor_ms_at_timed_sclk"] == pytest.approx(want_s, abs=1e-4)
    assert step["frac_at_timed_sclk"] > floor["frac_at_timed_sclk"]
    assert "burst_final_kernel" in step["kernels"]


def test_single_kernel_step_has_no_step_floor(joined):
    roof, valu = joined(_pmc(step=False))
    assert roof["traffic"] is not None
    assert "step" not in valu["issue_floor"]


def test_counters_at_another_clock_are_refused(joined):
    # a throttled profile box: 2.25 GHz under the PMC passes, 2.38 timed
    roof, valu = joined(_pmc(clock_ghz=2.25))
    assert roof["traffic"] is None and valu is None
    assert "MHz" in roof["traffic_note"] and "not joined" in roof["traffic_note"]
    # within 3 %: joined
    roof, _ = joined(_pmc(clock_ghz=2.33))
    assert roof["traffic"] == 1.5e9


def test_counters_of_another_build_are_refused(joined):
    roof, valu = joined(_pmc(build="fedcba9876543210"), fresh=False)
    assert roof["traffic"] is None and valu is None
    assert "fedcba9876543210" in roof["traffic_note"]


def test_no_counters_file(joined):
    roof, valu = joined(None, fresh=None)
    assert roof["traffic"] is None and valu is None
    # the algorithmic side is there regardless
    assert roof["frac"] == pytest.approx(815e6 / 0.7155e-3 / 1e9 / 8000, abs=1e-4)


def test_trace_box_at_another_clock_is_refused(joined):
    """The kernel trace committed beside the counters must come from a box
    that timed the config within 3 % of this line's clock (VERDICT round 5,
    item 5): the PMC clock alone agreeing is not enough."""
    pmc = _pmc()
    pmc["trace_box"]["sclk_mhz_during_timed_steps"] = 2250
    pmc["trace_avg_ns"] = 790_100.0
    roof, valu = joined(pmc)
    assert roof["traffic"] is None and valu is None
    assert "trace box" in roof["traffic_note"]
    pmc["trace_box"]["sclk_mhz_during_timed_steps"] = 2330
    roof, _ = joined(pmc)
    assert roof["traffic"] == 1.5e9
    assert roof["trace_kernel_ms"] == pytest.approx(0.7901)


def test_line_tail_keeps_every_config():
    """finalize_line: prose moves to one notes object, the contract's fields
    stay, and the closing summary carries every config's numbers, so the
    last ~2 KB of the printed line hold C3 / C4."""
    import json
    line = {"metric": "m", "value": 1.0, "unit": "digests/s", "n_gpus": 1,
            "ms_per_step": 0.6, "config": {"workload": "w" * 100},
            "roofline": {"frac": 0.22, "kernel_ms": 0.61},
            "cpu_baseline": {"value": 7.7e6, "unit": "digests/s", "cores": 16,
                             "kind": "port", "sample": "s" * 300,
                             "openssl_context": {"note": "n" * 200, "value": 1.0}},
            "extra_configs": {
                "c3": {"value": 2.28e9, "ms_per_step": 0.46, "metric": "x" * 120,
                       "roofline": {"frac": 0.209, "kernel_ms": 0.455,
                                    "traffic_over_algorithmic": 1.54},
                       "cpu_baseline": {"value": 1.1e7, "sample": "y" * 200}},
                "c4": {"value": 1.36e9, "ms_per_step": 0.77,
                       "roofline": {"frac": 0.185, "kernel_ms": 0.771}},
                "burst_rx_e2e": {"value": 7.2e7, "ms_per_step": 14.4,
                                 "pageable": {"value": 6.9e7}}}}
    out = bench.finalize_line(line)
    text = json.dumps(out)
    tail = text[-2000:]
    for want in ('"c3": {"value": 2280000000.0', '"frac": 0.209', '"c4"',
                 '"burst_rx_e2e"'):
        assert want in tail, want
    assert list(out)[-1] == "summary"
    assert out["cpu_baseline"]["sample"] == "s" * 300          # contract field kept
    assert "extra_configs.c3.metric" in out["notes"]
    assert "cpu_baseline.openssl_context.note" in out["notes"]
    assert list(out).index("notes") < list(out).index("roofline")

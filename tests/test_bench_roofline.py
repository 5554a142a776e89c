"""bench.py's roofline accounting on CPU (no GPU, no library): the primary entry's bytes and
PMC traffic are one step's when the step's wall time is the divisor, whatever the number of
segments a launch carries."""
import importlib

import pytest

bench = importlib.import_module("bench")


def fake_pmc(per_launch: dict, fpl: int):
    """load_pmc's shape: per-kernel HBM bytes per frame from a count of `fpl`-frame launches."""
    return {k: {"hbm_bytes_per_launch": v, "hbm_bytes_per_frame": v / fpl} for k, v in per_launch.items()}


@pytest.fixture
def workload():
    saved = (bench.W, bench.H, bench.DW, bench.DH)
    yield
    bench.W, bench.H, bench.DW, bench.DH = saved


def set_wl(name):
    bench.W, bench.H, bench.DW, bench.DH = bench.WORKLOADS[name][:4]


def test_default_primary_traffic_is_per_step(workload):
    set_wl("c2")
    seg = 120
    pmc = fake_pmc({"void mjg::k_encode<true, 0, false, false>": 1.9e9, "mjg::k_write": 8e7}, seg)
    kt = {"encode": 2.0, "scale": 0.0, "huff": 0.0}
    primary, ents = bench.rooflines(kt, 2 * seg, 322e3, pmc, False, False, step_ms=0.6, seg=seg)
    assert ents[0]["traffic"] == round(2 * 1.9e9)          # per 2-segment launch
    assert primary["traffic"] == round(1.9e9)              # per step (one segment)
    alg = bench.frame_bytes(3840, 2160) * seg + 322e3 * seg
    assert primary["alg_bytes_per_launch"] == int(alg)
    assert primary["frac"] == pytest.approx(alg / 0.6e-3 / 1e9 / 8000, abs=1e-4)


def test_optimal_primary_traffic_is_per_step(workload):
    set_wl("c1")
    seg = 250
    pmc = fake_pmc({"void mjg::k_encode<true, 1, false, false>": 1.39e9, "mjg::k_huff_build": 2e6,
                    "mjg::k_emit_syms": 5.2e8, "mjg::k_write": 4e7}, seg)
    kt = {"encode": 0.4, "scale": 0.0, "huff": 0.9}
    primary, ents = bench.rooflines(kt, 2 * seg, 75e3, pmc, True, False, step_ms=0.5, seg=seg)
    assert primary["traffic"] == round(1.39e9 + 2e6 + 5.2e8)
    # the per-kernel entries stay per launch
    assert ents[1]["traffic"] == round(2 * 5.2e8)
    # without a step time the primary is the launch's own
    p2, _ = bench.rooflines(kt, seg, 75e3, pmc, True, False)
    assert p2["traffic"] == round(1.39e9 + 2e6 + 5.2e8)


def test_scaled_primary_traffic_is_k_scale_plus_k_encode(workload):
    set_wl("c4")
    seg = 120
    pmc = fake_pmc({"void mjg::k_scale<8, 5, true, 1, 64>": 1.25e9, "void mjg::k_scale<8, 5, true, 2, 64>": 6.25e8,
                    "void mjg::k_encode<false, 0, false, false>": 5.09e8, "mjg::k_write": 3.4e7}, seg)
    kt = {"encode": 0.5, "scale": 1.0, "huff": 0.0}
    primary, ents = bench.rooflines(kt, 2 * seg, 100e3, pmc, False, True, step_ms=0.7, seg=seg)
    assert primary["traffic"] == round(1.25e9 + 6.25e8 + 5.09e8)
    assert ents[0]["kernel"] == "k_scale" and ents[0]["traffic"] == round(2 * (1.25e9 + 6.25e8))


def test_no_pmc_gives_null_traffic(workload):
    set_wl("c2")
    primary, ents = bench.rooflines({"encode": 1.0, "scale": 0.0, "huff": 0.0}, 240, 3e5, {}, False, False,
                                    step_ms=0.6, seg=120)
    assert primary["traffic"] is None and ents[0]["traffic"] is None


def test_gpus_without_launcher_runs_the_driver_launch_line():
    """`python bench.py --gpus N` outside torchrun re-runs itself under the driver's launch line
    (one rank per GPU, rendezvous on 127.0.0.1) as a child, with the same arguments."""
    argv = bench.torchrun_argv(4, ["--gpus", "4", "--steps", "5"], 29511)
    assert argv[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in argv and "--nnodes=1" in argv
    assert argv[argv.index("--master-addr") + 1] == "127.0.0.1"
    assert argv[argv.index("--master-port") + 1] == "29511"
    assert argv[-5].endswith("bench.py") and argv[-4:] == ["--gpus", "4", "--steps", "5"]

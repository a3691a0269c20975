"""bench.py's host-side pieces on the CPU: the CPU-baseline leg in every ISA-L
kernel family (the repair it times must rebuild D0 exactly), the leg
estimates and the rocprof-CSV roofline recomputation."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
import oracle  # noqa: E402


@pytest.mark.parametrize("kind", ["avx2", "avx512", "gfni"])
def test_cpu_stripe_every_family_rebuilds_d0(kind):
    if not oracle.Oracle().have_kind(kind):
        pytest.skip(f"no {kind} on this CPU")
    a = bench.parse([])
    res, ok = bench.cpu_stripe(a, 32, 2, 8, 1 << 16, [1, 2], 0.05, kind=kind)
    assert ok and res[1] > 0 and res[2] > 0


def test_cpu_baseline_reports_as_built_family():
    a = bench.parse(["--cpu-seconds", "0.2"])
    cb = bench.cpu_baseline(a, 32, 2, 8, 1 << 16)
    orc = oracle.Oracle()
    assert cb["isal_family"] == orc.isal_master_kind() and cb["kind"] == "port" and cb["cores"] == 1
    assert cb["value"] == cb["families_GBps"][cb["isal_family"]]["1"]
    for kind in ("avx2", "avx512", "gfni"):
        if orc.have_kind(kind):
            assert cb[f"value_{kind}"] > 0 and cb[f"value_{kind}_all_cores"] > 0


def test_profile_fracs_from_committed_csv(tmp_path):
    """The line's profile_frac is algorithmic bytes per launch / the most-called
    encode_kernel row's AverageNs / 8 TB/s (likewise the repair)."""
    csv = tmp_path / "stats.csv"
    csv.write_text('"Name","Calls","TotalDurationNs","AverageNs","Percentage"\n'
                   '"void encode_kernel_asm<1>(x)",86,1,5000000.0,1\n'
                   '"void encode_kernel_asm<2>(x)",2,1,9000000.0,1\n'
                   '"void xor_kernel_fixed<27, 4>(x)",43,1,2000000.0,1\n')
    a = bench.parse(["--profile-csv", str(csv)])
    p = bench.profile_fracs(a, 36_000_000_000, 16_000_000_000)
    assert p["profile_frac"] == round(36e9 / 5e-3 / 8e12, 4) and p["profile_encode_calls"] == 86
    assert p["profile_repair_frac"] == round(16e9 / 2e-3 / 8e12, 4)
    # another workload: no figure from a CSV taken on the default one
    a = bench.parse(["--profile-csv", str(csv), "--k", "32"])
    assert bench.profile_fracs(a, 1, 1)["profile_source"] is None


def test_default_profile_csv_is_committed():
    a = bench.parse([])
    assert os.path.exists(a.profile_csv)
    p = bench.profile_fracs(a, 36507222016, 15032385536)
    assert 0.7 < p["profile_frac"] < 1.0 and 0.7 < p["profile_repair_frac"] < 1.0


def test_leg_estimates_fit_the_budget_at_every_n():
    a = bench.parse([])
    for n in (1, 2, 4, 8):
        est = bench.leg_estimates(a, n)
        assert sum(est.values()) + 150 < a.budget_s < a.deadline_s  # 150 s: a slow first import + main leg

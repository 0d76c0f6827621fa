"""The capped spread tolerances of the driver-level parity tests (tests/spread_tol.py), on the
deviations measured on MI355X (tools/maps_spread.py, profiles/r05a/maps_spread.json): a focal
perturbed by 1e-2 px fails where the caps apply, every exemption is tied to its flow and message,
and an exemption whose premise no longer holds fails as stale."""
import pytest

from spread_tol import CAPS, EXEMPT, tolerance

# (device - oracle, alt - oracle) of the converged cfg1 map solve, focal in px (r05 measurement)
MAP_CFG1_FOCAL = (1.97e-6, 1.62e-6)
F = 901.0


def test_measured_deviations_pass():
    assert MAP_CFG1_FOCAL[0] <= tolerance("focal", F, F + MAP_CFG1_FOCAL[1])
    # the final cfg1 message: 2.6e-4 px both ways, under the 1e-3 px cap
    assert 2.6e-4 <= tolerance("focal", F, F + 2.59e-4, ("cfg1_incremental", 2))


def test_perturbed_focal_fails_under_the_cap():
    """1e-2 px of focal fails on a converged solve even where the arithmetics' spread is wide (the
    old uncapped 20x rule allowed ~1 px on cfg1)."""
    for alt_spread in (1.62e-6, 2.6e-4, 0.05):
        assert 1e-2 > tolerance("focal", F, F + alt_spread), alt_spread
    assert tolerance("focal", F, F + 0.05) == CAPS["focal"]


def test_exemptions_are_named_and_asserted():
    assert tolerance("focal", F, F + 0.048, ("cfg1_incremental", 0)) == pytest.approx(20 * 0.048)
    assert all(len(why) > 40 for why in EXEMPT.values())
    with pytest.raises(AssertionError, match="stale exemption"):
        tolerance("focal", F, F + 1e-6, ("cfg1_incremental", 0))   # the arithmetics agree: no reason left
    # a non-exempt message of the same flow stays capped
    assert tolerance("focal", F, F + 0.048, ("cfg1_incremental", 2)) == CAPS["focal"]


def test_centres_and_cost_caps():
    assert tolerance("centres", 1.0, 1.0 + 0.01) == CAPS["centres"]
    assert tolerance("centres", 1.0, 1.0) == 1e-5
    assert tolerance("cost", 100.0, 100.0 + 1.0) == pytest.approx(CAPS["cost"] * 100.0)

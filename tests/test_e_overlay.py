"""Config E's overlay after churn (tests/e_overlay.py):
size-independent properties of the live nodes outside the giant component,
on the oracle here and on the GPU at 2^18 nodes.

  * every one of them is a churn victim (crashed, restarted, rejoined);
  * most lost their rejoin to the partition: the JOIN crossed the half/half
    split while it was on, was dropped, and HyParView never retries a join
    (hv:500-515 sends it once; the restarted node's views are empty, so
    neither random_promotion nor a shuffle can bring it back);
  * the rest hang off those (rejoined through a contact outside the giant);
  * the fraction is stable after churn (same count at +49 and +89 rounds);
  * a broadcast after the churn reaches the whole giant component within
    20 rounds (Plumtree reliability = the overlay's connectivity).
The bounds: outside <= lost joins (every outside node is explained by one
lost join, directly or through its contact) and >= 60% lost-join nodes.

With the partition where SURVEY 8(d) E puts it -- phase rounds 150-169,
after the churn (schedule "survey", bench.py --workload E's default) -- no
rejoin meets it: the overlay heals to one component within 49 rounds of the
last rejoin and a broadcast then reaches every live node."""
import pytest

import e_overlay as E
from _oracle import Oracle


def check(rows, rel):
    a, b = rows[1], rows[2]                       # +49, +89
    for r in rows:
        assert r["outside_victims"] == r["outside"], r
        assert r["outside"] <= r["lost_joins"], r
        assert r["outside_lost_join"] >= 0.6 * r["outside"], r
    assert abs(a["outside"] - b["outside"]) <= max(2, a["outside"] // 50), (a, b)
    assert rel["delivered_20"] >= b["giant"] / b["n_up"] - 1e-3, (rel, b)
    assert rel["delivered_40"] == rel["delivered_20"], rel


def test_e_overlay_oracle():
    rows, rel = E.run(Oracle, 4096)
    check(rows, rel)


@pytest.mark.gpu
def test_e_overlay_gpu():
    from partisan_amd import Simulator
    rows, rel = E.run(Simulator, 1 << 18)
    check(rows, rel)
    assert rows[-1]["outside_frac"] < 0.03, rows[-1]


def check_survey(rows, rel):
    for r in rows:
        assert r["lost_joins"] == 0 and r["outside_victims"] == r["outside"], r
        assert r["outside_frac"] < 0.002, r
    assert rows[1]["outside"] == 0 and rows[2]["outside"] == 0, rows
    assert rel["delivered_20"] == 1.0 and rel["delivered_40"] == 1.0, rel


def test_e_overlay_survey_oracle():
    rows, rel = E.run(Oracle, 16384, schedule="survey")
    check_survey(rows, rel)


@pytest.mark.gpu
def test_e_overlay_survey_gpu():
    from partisan_amd import Simulator
    rows, rel = E.run(Simulator, 1 << 18, schedule="survey")
    check_survey(rows, rel)

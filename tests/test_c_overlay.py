"""Config C's overlay on the survey schedule (tests/c_overlay.py; VERDICT r3
item 6): size-independent properties of the live nodes outside the giant
component, on the oracle here (2^14: none) and on the GPU at 2^18 and 2^20.

  * none is isolated -- each sits in a closed component of >= 2 nodes and
    holds >= 2 active peers, at or above min_active_size (3 with the node
    itself): random_promotion never fires for it (hv:542-556, :1718-1728);
  * the outside set forms during the join ramp and is the same set of nodes
    from 16 rounds after the ramp's end through the bench's window;
  * the broadcast of the window reaches exactly the giant component;
  * the fraction stays small: below 0.2 % (46 nodes at 2^18, 902 at 2^20 --
    the oracle's counts, equal bit for bit on the GPU)."""
import pytest

import c_overlay as C
from _oracle import Oracle


def check(r, bound):
    rows, last = r["rows"], r["rows"][-1]
    assert last["isolated"] == 0, last
    assert last["outside"] == 0 or last["min_peers_outside"] >= 2, last
    assert last["outside_frac"] <= bound, last
    assert r["stable_since"] <= C.W.SURVEY_RAMP + 16, r["stable_since"]
    assert abs(last["delivered_frac"] - last["giant"] / last["n_up"]) < 1e-9, last
    assert all(x == 0 or x >= 2 for x in last["comp_sizes"]), last
    return last


def test_c_overlay_oracle():
    last = check(C.run(Oracle, 1 << 14), 0.002)
    assert last["outside"] == 0, last


@pytest.mark.gpu
@pytest.mark.parametrize("n,outside", [(1 << 18, 46), (1 << 20, 902)])
def test_c_overlay_gpu(n, outside):
    from partisan_amd import Simulator
    last = check(C.run(Simulator, n), 0.002)
    assert last["outside"] == outside, last

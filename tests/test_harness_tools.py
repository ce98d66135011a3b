"""The harness comparison tool (erlang/harness/compare_trace.py) on CPU:
its scenario files and the oracle's record stream are well formed, the
stream is deterministic, and compare() flags the first differing record.
The Erlang side itself cannot run here (no Erlang VM)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "erlang", "harness", "compare_trace.py")


def _run(*a):
    return subprocess.run([sys.executable, TOOL] + list(a), capture_output=True, text=True, timeout=300)


def test_scenario_and_compare(tmp_path):
    d = str(tmp_path)
    r = _run("scenario", "doubling_crash_256", d)
    assert r.returncode == 0, r.stderr
    terms = open(os.path.join(d, "doubling_crash_256.terms")).read()
    assert terms.startswith("{config, #{n_nodes => 256") and "{crash, 40, [5, 22" in terms
    stream = os.path.join(d, "doubling_crash_256.oracle")
    head, *lines = open(stream).read().splitlines()
    assert head == "S doubling_crash_256"
    assert len(lines) > 1000 and all(l.startswith("R ") for l in lines)
    # (src, seq) numbering: per round and source, seq runs 0, 1, 2, ...
    seen = {}
    for l in lines:
        f = l.split()
        key = (f[1], f[2])
        assert int(f[3]) == seen.get(key, -1) + 1
        seen[key] = int(f[3])
    assert _run("compare", stream, stream).returncode == 0
    bad = os.path.join(d, "bad")
    mod = [head] + lines
    mod[501] = mod[501].rsplit(" ", 1)[0] + " 999"
    open(bad, "w").write("\n".join(mod) + "\n")
    r = _run("compare", bad, stream)
    assert r.returncode == 1 and "record 500 differs" in r.stdout


def test_strategy_scenarios(tmp_path):
    """The pluggable-manager scenarios of psim_strategy_harness.erl (configs
    B and D in miniature): the event script names the strategy, its leave/1
    and partition events, and the oracle's stream carries the handshake and
    the strategy's own message types in the harness's record format."""
    d = str(tmp_path)
    for name, types in (("scamp_v1_128_pl", {0, 1, 3, 4, 6}), ("scamp_v2_128_pl", {0, 1, 3, 4, 5, 7}),
                        ("full_16_pl", {0, 1, 2})):
        r = _run("scenario", name, d)
        assert r.returncode == 0, r.stderr
        terms = open(os.path.join(d, name + ".terms")).read()
        strategy = name.rsplit("_", 2)[0] if name.startswith("full") else name[:8]
        assert f"strategy => {strategy}" in terms and "periodic_interval => 10" in terms
        if name.startswith("scamp"):
            assert "{leave, 50, [{9, 10}]}." in terms and "{clear_partition, 70}." in terms
        lines = [l for l in open(os.path.join(d, name + ".oracle")).read().splitlines() if l.startswith("R ")]
        got = {int(l.split()[5]) for l in lines}
        assert types <= got, (name, sorted(got))
        assert all(len(l.split()) == 11 and l.split()[6] == "0" for l in lines)   # ttl 0, no exchange ids
        assert _run("compare", os.path.join(d, name + ".oracle"), os.path.join(d, name + ".oracle")).returncode == 0


def test_compare_takes_the_harness_bucket_table(tmp_path):
    """App. A Q1: the harness writes erlang:phash(NodeSpec, 16) of every node
    (`B id bucket`); compare regenerates the oracle stream with that table
    (psim_set_bucket_table) before diffing, so a harness run whose sets order
    is not the oracle's stand-in still compares record for record.  Here the
    "harness output" is the oracle's own stream under a random table."""
    sys.path.insert(0, os.path.dirname(TOOL))
    import compare_trace as CT
    import numpy as np
    import _scenarios as S
    d = str(tmp_path)
    assert _run("scenario", "config_a", d).returncode == 0
    default = os.path.join(d, "config_a.oracle")
    tab = S.random_buckets(32, 5)
    fake = os.path.join(d, "config_a.harness")
    CT.write_stream("config_a", fake, tab)
    assert open(fake).read().count("\nB ") == 32
    r = _run("compare", fake, default)
    assert r.returncode == 0 and "regenerated" in r.stdout and "records identical" in r.stdout, r.stdout
    assert np.array_equal(CT.read_buckets(os.path.join(d, "bucket16.txt"), 32), tab)
    # the default stream differs from the table's: without the table the diff fails
    h = [l for l in open(fake) if l.startswith("R ")]
    o = [l for l in open(default) if l.startswith("R ")]
    assert h != o
    plain = os.path.join(d, "plain.harness")
    open(plain, "w").writelines(h)
    assert _run("compare", plain, default).returncode == 1
    # a scenario made with the table from the start compares without regenerating
    bt = os.path.join(d, "tab.txt")
    open(bt, "w").write("".join(f"{i} {int(b)}\n" for i, b in enumerate(tab)))
    assert _run("scenario", "config_a", d, bt).returncode == 0
    r = _run("compare", fake, default)
    assert r.returncode == 0 and "regenerated" not in r.stdout

# debug: GPU config A after a pluggable-manager run in the same process
import sys; sys.path[:0] = ['.', 'tests']
import _scenarios as S
from partisan_amd import Simulator
from _oracle import Oracle
mode = sys.argv[1] if len(sys.argv) > 1 else "pl"
if mode == "pl":
    S.pl_doubling(lambda c: Simulator(c), 1 << 12, 13, 30, strategy=2)
elif mode == "full":
    S.pl_doubling(lambda c: Simulator(c), 1024, 11, 30, strategy=0, fanout=5)
elif mode == "hv":
    S.doubling(lambda c: Simulator(c), 1024, 1, 30)
g, gst = S.config_a(lambda c: Simulator(c))
o, ost = S.config_a(Oracle)
print(mode, "gpu emitted", gst['emitted'].sum(1)[:6], "digest", gst['digest'][:3], "proc", gst['nodes_processed'][:6])
print(mode, "orc emitted", ost['emitted'].sum(1)[:6], "digest", ost['digest'][:3], "proc", ost['nodes_processed'][:6])

import sys, os
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, p) for p in ('uigc-akka_amd', 'tests', 'workload', 'oracle')]
os.environ['CRGC_DEBUG_GATHER'] = '1'
import kats, oracle, crgc_hip
w = kats.RandomWorld(seed=7, max_actors=600, wake_every=13)
b = next(iter(w.steps()))
parts = b.split(4)
h = crgc_hip.ShardedShadowGraph(4)
h._all(lambda s, x: s.merge_entries(x), [(p,) for p in parts])
print(sorted(h.shards[0].export().vertices), flush=True)

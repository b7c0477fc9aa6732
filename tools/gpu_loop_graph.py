"""Run test_graph_replay_matches_eager N times in one process (flakiness probe)."""
import os, sys
root = sys.argv[1]
n = int(sys.argv[2])
sys.path[:0] = [os.path.join(root, "tests"), root, os.path.join(root, "ceo-recommender_amd")]
os.chdir(root)
import test_gpu_parity as T
fails = 0
for i in range(n):
    try:
        T.test_graph_replay_matches_eager(False)  # atomic mode: the optimizer-scale bound
        print(f"{root} run {i}: ok", flush=True)
    except AssertionError as e:
        fails += 1
        print(f"{root} run {i}: FAIL {str(e)[:120]}", flush=True)
print(f"{root}: {fails}/{n} failed", flush=True)

"""Same-process A/B of the light / heavy split (capi.cpp split_rows) on C5 at 10M requests: the
unsplit upload against split uploads under heavy thresholds (KW_HEAVY_CTR, at upload) and
heavy-region tile heights (KW_HEAVY_ROWS, at planning), each timed with HIP events around the pass
(kw_validate_timed), interleaved over rounds.
Run on the GPU box: CFGS="16:24,12:24" python scripts/split_ab.py [rows] [rounds]
(a config is heavy_ctr:heavy_rows; heavy_rows 0 plans the heavy region like any batch)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "policy-server_amd"), os.path.join(ROOT, "tests")]
import kwgpu as K  # noqa: E402
from helpers import config  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    cfgs = [tuple(c.split(":")) for c in os.environ.get("CFGS", "16:0,16:24").split(",")]
    env = K.EvaluationEnvironment(config("c5_mixed"), continue_on_errors=True, always_accept_namespace="kubewarden",
                                  device=0)
    ids = env.policy_ids()
    t0 = time.time()
    syn = K.SynthBatch(5, n, seed=5)
    print(f"[split_ab] generated {n} rows in {time.time() - t0:.1f} s", flush=True)
    os.environ["KW_SPLIT"] = "0"
    batches = {"unsplit": (syn.batch().to_device(0), "0")}
    os.environ["KW_SPLIT"] = "1"
    for ctr in sorted({c for c, _ in cfgs}):
        os.environ["KW_HEAVY_CTR"] = ctr
        t0 = time.time()
        batches[ctr] = (syn.batch().to_device(0), ctr)
        print(f"[split_ab] split upload (heavy > {ctr} containers) {time.time() - t0:.1f} s", flush=True)
    res = {}
    for r in range(rounds):
        os.environ.pop("KW_HEAVY_ROWS", None)
        res.setdefault("unsplit", []).append(batches["unsplit"][0].timed(env, ids, warmup=2, reps=10).evaluate_ms)
        for ctr, rows in cfgs:
            if rows == "0":
                os.environ.pop("KW_HEAVY_ROWS", None)
            else:
                os.environ["KW_HEAVY_ROWS"] = rows
            t = batches[ctr][0].timed(env, ids, warmup=2, reps=10)
            res.setdefault(f"split heavy>{ctr} rows={rows}", []).append(t.evaluate_ms)
        print(f"[split_ab] round {r}: " + ", ".join(f"{k} {v[-1]:.3f}" for k, v in res.items()), flush=True)
    for k, v in res.items():
        print(f"{k}: median {sorted(v)[len(v) // 2]:.3f} ms  all {[round(x, 3) for x in v]}")


if __name__ == "__main__":
    main()

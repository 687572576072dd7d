"""Bulk path (kw_validate_host) knob sweep on the GPU box: C4 1M x 64 into a pinned verdict buffer,
best of 7, one process per setting (the knobs are read once per process). Usage:
KW_BULK_DEPTH=4 python scripts/bulk_knobs.py [rows]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "policy-server_amd"), os.path.join(ROOT, "tests")]
import kwgpu as K  # noqa: E402
from helpers import config  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    env = K.EvaluationEnvironment(config("c4_64"), continue_on_errors=True, always_accept_namespace="kubewarden", device=0)
    ids = env.policy_ids()
    syn = K.SynthBatch(4, n, seed=4)
    pin = K.PinnedWords(n * len(ids))
    best = 1e9
    for _ in range(8):
        hb = syn.batch()
        t0 = time.perf_counter()
        hb.validate_host(env, ids, out=pin.array)
        best = min(best, time.perf_counter() - t0)
        hb.close()
    knobs = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("KW_BULK"))
    print(f"{knobs or 'default'}: best {best * 1e3:.2f} ms = {n / best / 1e6:.1f} M req/s", flush=True)


if __name__ == "__main__":
    main()

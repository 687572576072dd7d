"""Single-thread flatten rate (kw_batch_from_json, AdmissionReview JSON -> SoA columns) on synthetic
workload documents: best of --reps timed calls over --n documents, one JSON line per config."""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "policy-server_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="4,5")
    ap.add_argument("--n", type=int, default=50_000)
    ap.add_argument("--reps", type=int, default=7)
    args = ap.parse_args()
    import kwgpu as K
    os.environ["KW_FLATTEN_THREADS"] = "1"
    L = K._native.lib()
    for cfg in [int(c) for c in args.configs.split(",")]:
        syn = K.SynthBatch(cfg, args.n, seed=20250509)
        docs = [syn.json(i).encode() for i in range(args.n)]
        arr = (C.c_char_p * args.n)(*docs)
        lens = (C.c_size_t * args.n)(*[len(d) for d in docs])
        best = 1e9
        for _ in range(args.reps):
            h, bad, err = C.c_void_p(), C.c_int64(-1), C.create_string_buffer(512)
            t = time.perf_counter()
            rc = L.kw_batch_from_json(arr, lens, args.n, K._native.KW_DOC_ADMISSION_REVIEW, C.byref(h), C.byref(bad), err, len(err))
            best = min(best, time.perf_counter() - t)
            assert rc == 0, err.value
            L.kw_batch_destroy(h)
        nb = sum(len(d) for d in docs)
        print(json.dumps({"config": cfg, "requests_per_s_per_thread": args.n / best, "GB_per_s": nb / best / 1e9,
                          "mean_doc_bytes": nb / args.n}), flush=True)


if __name__ == "__main__":
    main()

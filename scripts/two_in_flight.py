"""Two HBM-resident C4 passes in flight (bench.py timing_modes.two_in_flight), for a rocprofv3 kernel
trace: two device copies of the batch, each on its own stream, `--steps` passes alternating.
Run under: rocprofv3 --kernel-trace -d <dir> -o run --output-format csv -- python3 scripts/two_in_flight.py"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "policy-server_amd"), ROOT]

import torch  # noqa: E402
import yaml  # noqa: E402

import kwgpu as K  # noqa: E402
from bench import CONFIGS, SEED  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--config", default="c4_64")
args = ap.parse_args()
synth, rows, _ = CONFIGS[args.config]
with open(os.path.join(ROOT, "configs", f"{args.config}.yml")) as f:
    env = K.EvaluationEnvironment(yaml.safe_load(f), device=0)
ids = env.policy_ids()
syn = K.SynthBatch(synth, rows, seed=SEED)
ba, bb = syn.batch().to_device(0), syn.batch().to_device(0)
for b in (ba, bb, ba, bb):
    b.validate(env, ids)
torch.cuda.synchronize()
t = time.perf_counter()
for i in range(args.steps):
    (ba if i % 2 == 0 else bb).validate(env, ids)
torch.cuda.synchronize()
dt = time.perf_counter() - t
print(f"[two] {args.steps} passes of {rows} rows in {dt * 1e3:.3f} ms: {rows * args.steps / dt / 1e9:.3f} G req/s")

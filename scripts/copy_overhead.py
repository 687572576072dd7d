import torch, time
dev = torch.device("cuda:0")
total = 168 << 20
h = torch.empty(total, dtype=torch.uint8).pin_memory()
d = torch.empty(total, dtype=torch.uint8, device=dev)
s = torch.cuda.Stream()
def run(npieces, reps=5):
    best = 1e9
    step = total // npieces
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            for i in range(npieces):
                d[i*step:(i+1)*step].copy_(h[i*step:(i+1)*step], non_blocking=True)
        s.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3
for n in [1, 11, 55, 110, 220, 440]:
    ms = run(n)
    print(f"{n:4d} pieces: {ms:.3f} ms  {total/ms/1e6:.1f} GB/s  per-piece overhead vs 1: {(ms - run(1))/max(n-1,1)*1e3:.1f} us")

"""Overlap of the tile kernels in a rocprofv3 kernel trace (scripts/two_in_flight.py): per kernel its
duration, and the union of all tile-kernel intervals against their sum."""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "evaluate_tiles" in r["Kernel_Name"]]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id", r.get("Queue_Id", "?"))) for r in rows)
iv = iv[4:]  # the warm-up passes
total = sum(e - s for s, e, _ in iv)
union, cur_s, cur_e = 0, None, None
for s, e, _ in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            union += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
union += cur_e - cur_s
span = iv[-1][1] - iv[0][0]
print(f"kernels {len(iv)}, mean duration {total / len(iv) / 1e3:.1f} us, sum {total / 1e3:.1f} us, "
      f"busy union {union / 1e3:.1f} us, span {span / 1e3:.1f} us, overlap {1 - union / total:.1%}")
for s, e, q in iv[:6]:
    print(f"  start {(s - iv[0][0]) / 1e3:9.1f} us  end {(e - iv[0][0]) / 1e3:9.1f} us  stream/queue {q}")

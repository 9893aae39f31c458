"""Summarise a rocprofv3 --kernel-trace CSV of a bench run: per-kernel time per training step over the
last timed steps (each step from its input quantiser's first launch to its NITI_SGD update launch and the fused
fully connected updates after it),
then the last step's launches as a timeline.  Launches outside those steps (autotuning, warmup, the
isolated probe re-runs after the timed region) are not counted.

usage: prof_summary.py kernel_trace.csv [steps]   (steps: how many of the last steps to average)
"""
import collections
import csv
import sys

path = sys.argv[1]
want = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # noqa: E731


def short(n):
    n = n.replace("(anonymous namespace)::", "").split("(")[0].replace("void niti::", "").replace("niti::", "")
    return n.replace("gemm_i8_kernel", "gemm").replace("Load", "")[:80]


def is_start(r):  # a step's first kernel: the input statistics or the int8 input's relayout / im2col
    k = r["Kernel_Name"]
    return "image_stats" in k or "NchwToNhwc16" in k or "input_im2col" in k


def is_update_tail(r):  # the fully connected layers' fused NITI_SGD passes follow the update launch
    return "KtRowsU, niti::KtRowsU, 4, true" in r["Kernel_Name"]


# steps: [start index, index of the sgd_update launch or the last fused-update pass after it]; the
# stats launch may be preceded by a memset
ends = []
for i, r in enumerate(rows):
    if "sgd_update_kernel" in r["Kernel_Name"]:
        while i + 1 < len(rows) and is_update_tail(rows[i + 1]):
            i += 1
        ends.append(i)
steps = []
prev = -1
for e in ends:
    s = min((i for i in range(prev + 1, e) if is_start(rows[i])), default=None)
    prev = e
    if s is None:
        continue
    steps.append((s, e))
steps = steps[-want:]
if not steps:
    sys.exit("no complete step in the trace")
tot = collections.defaultdict(float)
cnt = collections.Counter()
for s, e in steps:
    for r in rows[s:e + 1]:
        tot[short(r["Kernel_Name"])] += dur(r)
        cnt[short(r["Kernel_Name"])] += 1
n = len(steps)
print(f"per-kernel time per step, averaged over the last {n} steps")
print(f"{'us/step':>9} {'calls/step':>10}  kernel")
for k, v in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"{v / n:9.1f} {cnt[k] / n:10.1f}  {k}")
busy = sum(tot.values()) / n
span = sum((int(rows[e]["End_Timestamp"]) - int(rows[s]["Start_Timestamp"])) / 1e3 for s, e in steps) / n
print(f"busy us/step {busy:.1f}   first launch -> update end us/step {span:.1f}   launches/step "
      f"{sum(cnt.values()) / n:.1f}")
s, e = steps[-1]
seg = rows[s:e + 1]
t0 = int(seg[0]["Start_Timestamp"])
print("\nlast step's launches:")
print(f"{'start':>8} {'dur':>7} {'gap':>6}  grid        kernel")
prev_end = t0
for r in seg:
    st = int(r["Start_Timestamp"])
    grid = f"{r.get('Grid_Size_X', r.get('Grid_Size', '?'))}"
    print(f"{(st - t0) / 1e3:8.2f} {dur(r):7.2f} {max(0, st - prev_end) / 1e3:6.2f}  {grid:<10}  {short(r['Kernel_Name'])}")
    prev_end = max(prev_end, int(r["End_Timestamp"]))

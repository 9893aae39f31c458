"""Summarise a rocprofv3 --kernel-trace CSV: per-kernel totals per step and the last step's launches."""
import collections
import csv
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 13
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # noqa: E731


def short(n):
    n = n.split("(")[0].replace("void niti::", "").replace("niti::", "")
    return n.replace("gemm_i8_kernel", "gemm").replace("Load", "")[:70]


tot = collections.defaultdict(float)
cnt = collections.Counter()
for r in rows:
    tot[short(r["Kernel_Name"])] += dur(r)
    cnt[short(r["Kernel_Name"])] += 1
print(f"{'us/step':>9} {'calls/step':>10}  kernel")
for k, v in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"{v / steps:9.1f} {cnt[k] / steps:10.1f}  {k}")
print("total busy us/step", sum(tot.values()) / steps)
# last step: from the last loss_grad to the end
def is_start(r):  # a step's first kernel: the input quantiser or the int8 input's relayout
    return "image_stats" in r["Kernel_Name"] or "NchwToNhwc16" in r["Kernel_Name"]


idx = max(i for i, r in enumerate(rows) if "loss_grad" in r["Kernel_Name"])
first = max(i for i, r in enumerate(rows[:idx]) if is_start(r))
print("\nlast step launches (from the forward of the step):")
seg = rows[first:]
span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
t0 = int(seg[0]["Start_Timestamp"])
qcol = "Queue_Id" if "Queue_Id" in seg[0] else ("Stream_Id" if "Stream_Id" in seg[0] else None)
last_end = {}
print(f"{'start':>8} {'dur':>7} {'gap':>6}  q  grid        kernel")
for r in seg:
    g = f"{int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])}x{r['Grid_Size_Y']}"
    q = r[qcol] if qcol else "-"
    s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s0 - last_end[q]) / 1e3 if q in last_end else 0.0
    last_end[q] = e0
    print(f"{(s0 - t0) / 1e3:8.2f} {dur(r):7.2f} {gap:6.2f} {q:>2}  {g:>10}  {short(r['Kernel_Name'])}")
print("step span us", span, "busy", sum(dur(r) for r in seg), "launches", len(seg))

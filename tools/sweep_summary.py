"""Group the GEMM / reduce dispatches of a rocprofv3 kernel trace by kernel and grid."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
order = []
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void niti::", "")[:60]
    key = (name, int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), int(r["Grid_Size_Y"]))
    if key not in d:
        order.append(key)
    d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k in order:
    v = sorted(d[k])
    med = v[len(v) // 2]
    print(f"{k[1]:6d}x{k[2]:<4d} n={len(v):3d} med {med:8.2f} us  min {v[0]:8.2f}  {k[0]}")

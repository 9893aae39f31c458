#!/usr/bin/env python3
"""Copy one round's GPU deliverables from gpurun_out/ (tools/gpu_full.sh) into profiles/.

usage: collect_profiles.py TAG   (reads gpurun_out/{bench_full,prof,pmcF,pmcW}_TAG)
Writes profiles/TAG_bench.json, TAG_vgg11_b256_bench_under_rocprof.json, TAG_vgg11_b256_kernel_stats.csv,
TAG_vgg11_b256_step_breakdown.txt, TAG_probe_dispatches.txt, TAG_pmc_{fetch,write}_size.csv (probe rows +
calibration), TAG_traffic.txt and profiles/traffic.json.
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles")


def line(path):
    return json.loads([x for x in open(path) if x.startswith("{")][-1])


def main():
    tag = sys.argv[1]
    bench = line(f"{G}/bench_full_{tag}.log")
    json.dump(bench, open(f"{P}/{tag}_bench.json", "w"))
    open(f"{P}/{tag}_bench.json", "a").write("\n")
    prof = line(f"{G}/prof_{tag}.log")
    json.dump(prof, open(f"{P}/{tag}_vgg11_b256_bench_under_rocprof.json", "w"))
    shutil.copy(glob.glob(f"{G}/prof_{tag}/*kernel_stats.csv")[0], f"{P}/{tag}_vgg11_b256_kernel_stats.csv")
    trace = glob.glob(f"{G}/prof_{tag}/*kernel_trace.csv")[0]
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof_summary.py"), trace, "20"],
                         capture_output=True, text=True, check=True).stdout
    open(f"{P}/{tag}_vgg11_b256_step_breakdown.txt", "w").write(
        "per-kernel totals cover the whole profiled process (autotuning candidates included);\n"
        "the timeline below is the last training step\n" + out)
    # probe dispatches in the profiled run: the probed kernel and grid, in-step vs isolated (last 20)
    plan = prof["roofline"]["plan"]
    name = "wgrad_taps_kernel" if plan["bm"] == 32 else "gemm_kernel"
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    blocks = 32 * plan["splits"] if plan["bm"] == 32 else None
    sel = [r for r in rows if name in r["Kernel_Name"] and (blocks is None or int(r["Grid_Size_X"]) == blocks * 512)]
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in sel]
    steps = prof["steps"] + prof["warmup"]
    instep, iso = d[-(20 + steps):-20], d[-20:]
    with open(f"{P}/{tag}_probe_dispatches.txt", "w") as f:
        f.write(f"probe: {sel[-1]['Kernel_Name'].split('(')[0]} grid {sel[-1]['Grid_Size_X']} work items, plan {plan}\n")
        f.write(f"in-step launches (warmup + timed, overlapped with the input-gradient stream): n={len(instep)} "
                f"avg {sum(instep) / len(instep):.2f} us min {min(instep):.2f} max {max(instep):.2f}\n")
        f.write(f"isolated launches (re-run alone after the timed region): n={len(iso)} "
                f"avg {sum(iso) / len(iso):.2f} us min {min(iso):.2f} max {max(iso):.2f}\n")
        f.write(f"bench under rocprof (HIP events): avg_launch_us {prof['roofline']['avg_launch_us']} (in-step), "
                f"{prof['roofline']['isolated']['avg_launch_us']} (isolated); in-kernel span "
                f"{prof['roofline'].get('in_kernel_span_us')} / {prof['roofline']['isolated'].get('in_kernel_span_us')}\n")
    print(open(f"{P}/{tag}_probe_dispatches.txt").read())
    # PMC: probe rows + calibration
    gx = blocks * 512 if blocks else 0
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "traffic.py"), f"{G}/pmcF_{tag}", f"{G}/pmcW_{tag}",
                          f"{P}/traffic.json", str(gx), "1", name, "20"], capture_output=True, text=True, check=True).stdout
    open(f"{P}/{tag}_traffic.txt", "w").write(out)
    print(out)
    for cnt, fn in (("pmcF", "fetch"), ("pmcW", "write")):
        src = glob.glob(f"{G}/{cnt}_{tag}/*counter_collection.csv")[0]
        rs = list(csv.DictReader(open(src)))
        keep = [r for r in rs if "NchwToNhwc16" in r["Kernel_Name"] or
                (name in r["Kernel_Name"] and int(r["Grid_Size"]) == gx)]
        with open(f"{P}/{tag}_pmc_{fn}_size.csv", "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rs[0].keys()))
            w.writeheader()
            w.writerows(keep)


if __name__ == "__main__":
    main()

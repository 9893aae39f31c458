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
    p16 = plan["bm"] == 16  # the P16 weight-gradient kernel (niti_wgrad.hip)
    name = "wgrad_p16_kernel" if p16 else "wgrad_taps_kernel" if plan["bm"] == 32 else "gemm_kernel"
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    blocks = 32 * plan["splits"] if plan["bm"] == 32 else None
    sel = [r for r in rows if name in r["Kernel_Name"] and (blocks is None or int(r["Grid_Size_X"]) == blocks * 512)]
    if p16:  # the probe's grid: the last 20 dispatches are the isolated re-runs
        gx_p16, kn_p16 = int(sel[-1]["Grid_Size_X"]), sel[-1]["Kernel_Name"]
        # same instantiation and grid (other P16 layers can share the grid: <2,4,4> / <4,4,4>)
        sel = [r for r in sel if int(r["Grid_Size_X"]) == gx_p16 and r["Kernel_Name"] == kn_p16]
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in sel]
    steps = prof["steps"] + prof["warmup"]
    instep, iso = d[-(20 + steps):-20], d[-20:]
    R, Rp = bench["roofline"], prof["roofline"]
    ops = R["ops_per_launch"]
    iso_avg = sum(iso) / len(iso)
    with open(f"{P}/{tag}_probe_dispatches.txt", "w") as f:
        kn = sel[-1]["Kernel_Name"].split("(")[0]
        f.write(f"probe {kn}, grid {int(sel[-1]['Grid_Size_X']) // int(sel[-1]['Workgroup_Size_X'])} x "
                f"{sel[-1]['Workgroup_Size_X']} threads, plan {plan}\n")
        f.write(f"rocprofv3 --kernel-trace of `bench.py --cpu-sample 0 --load-plans ...` (tools/gpu_full.sh, TAG={tag}):\n")
        f.write(f"  isolated re-runs after the timed region (last 20 dispatches): avg {iso_avg:.2f} us, "
                f"min {min(iso):.2f}, max {max(iso):.2f}\n")
        if instep:
            f.write(f"  in-step dispatches (warmup + timed): n={len(instep)} avg {sum(instep) / len(instep):.2f} us\n")
        f.write(f"same run, bench.py HIP events (under the profiler): in-step avg {Rp['avg_launch_us']} us, isolated avg "
                f"{Rp['isolated']['avg_launch_us']} us, in-kernel span {Rp.get('in_kernel_span_us')} us\n")
        f.write(f"ops per launch {ops}; at the rocprof isolated duration: {ops / iso_avg / 1e6:.1f} TOPS = "
                f"{ops / iso_avg / 1e6 / R['peak']:.3f} of {R['peak']:.0f} TOPS\n")
        f.write(f"unprofiled bench line ({tag}_bench.json): in-step {R['avg_launch_us']} us = {R['frac']:.4f} of peak, "
                f"isolated {R['isolated']['avg_launch_us']} us = {R['isolated']['frac']:.4f}\n")
    print(open(f"{P}/{tag}_probe_dispatches.txt").read())
    # PMC: probe rows + calibration
    gx = gx_p16 if p16 else blocks * 512 if blocks else 0
    # the plan the counters were collected under: bench.py reports the traffic only for that plan
    pl = ",".join(str(plan[k]) for k in ("bm", "bn", "splits", "strategy"))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "traffic.py"), f"{G}/pmcF_{tag}", f"{G}/pmcW_{tag}",
                          f"{P}/traffic.json", "vgg11_b256_L3_p2", pl], capture_output=True, text=True, check=True).stdout
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
    # every launch of the last step: HBM bytes (PMC) over its un-counted duration
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "membound.py"), f"{G}/pmcF_{tag}", f"{G}/pmcW_{tag}",
                        f"{G}/prof_{tag}", f"{P}/{tag}_step_hbm.txt"], capture_output=True, text=True)
    print(r.stdout or r.stderr)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Benchmark: NITI int8 training images/sec (+ int8 MFMA TOPS) on VGG-11, batch 256 per GPU.

A step is one full NITI_SGD training step of VGG-11 on a 3x32x32 int8 batch, entirely on
device: 9 NITI_Conv_Int8 forwards (+relu/maxpool), NITI_LOSS_Grad, 9 weight gradients,
8 input gradients, pool/relu gradients and the int8 weight update.  Data-parallel runs
(torchrun, one process per GPU) shard nothing else: each rank trains its own 256 images
and the exact-mode RCCL all-reduces (MAX of every range, SUM of every int32 weight
gradient) keep all ranks bit-identical to one device running the global batch.

Prints ONE JSON line on rank 0 (contract in the task statement).

Launch: `python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment starts the N
ranks itself (torch.distributed.run as a child process, 127.0.0.1 rendezvous, before anything
touches the GPU) and exits with its code; under torchrun the world size must equal --gpus.
`--global-batch G` holds the global batch fixed (G / N images per GPU, strong scaling, BASELINE
configs 4 and 5: 512 and 1024 on 8 GPUs); otherwise every GPU trains `--batch` images (weak).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mandheling-dsp-training_amd"))


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv):
    """Start `n` ranks of this script under torch.distributed.run (one process per GPU) as a
    child process and return its exit code.  Called before any GPU call in this process."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this pool (RCCL)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd, env=env)


def resolve_world(args):
    """(world, rank, local_rank) from the torchrun environment, checked against --gpus."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def per_gpu_batch(args, world, default):
    """Images per GPU: --global-batch / world (strong scaling), else --batch or the default (weak)."""
    if args.global_batch:
        if args.global_batch % world:
            raise SystemExit(f"bench.py: --global-batch {args.global_batch} is not a multiple of {world} GPUs")
        return args.global_batch // world, "strong"
    return (args.batch or default), "weak"


def parallelism_label(world, what):
    return f"dp{world} exact ({what})" if world > 1 else "single GPU"


def spawn_check(args):
    """--spawn-check (CPU, no GPU call): every rank joins a gloo group and all-reduces its rank;
    rank 0 prints the line's launch fields.  Exercises the self-launch path on a CPU box."""
    import torch
    import torch.distributed as dist
    world, rank, _ = resolve_world(args)
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.tensor([rank + 1], dtype=torch.int64)
    if world > 1:
        dist.all_reduce(t)
    b, scaling = per_gpu_batch(args, world, 256)
    if rank == 0:
        print(json.dumps({"n_gpus": world, "ranks_sum": int(t.item()), "per_gpu_batch": b,
                          "global_batch": b * world, "scaling": scaling,
                          "parallelism": parallelism_label(world, "spawn check")}), flush=True)
    if world > 1:
        dist.destroy_process_group()


PEAK_INT8_TOPS = 256 * 4 * 2048 * 2.4e9 / 1e12  # 256 CU x 4 SIMD x 2048 int8 op/clk x 2.4 GHz = 5033
PEAK_HBM_GBS = 8000.0
METRIC = "training images/sec + int8 MFMA TOPS, VGG-11 batch 256, 1/2/4/8 MI355X"


def synth_weights(layers, seed):
    import numpy as np
    rng = np.random.default_rng(seed)
    out = []
    for l in layers:
        shape = (l["c_out"], l["c_in"], l["kh"], l["kw"])
        fan_in = l["c_in"] * l["kh"] * l["kw"]
        fan_out = l["c_out"] * l["kh"] * l["kw"]
        t = rng.normal(0.0, (2.0 / (fan_in + fan_out)) ** 0.5, size=shape).astype(np.float32)
        r = float(np.abs(t).max())  # nn/Distributions.cpp:26-51 with a fixed seed
        out.append((np.round(t / r * 127).astype(np.int8), int(np.ceil(np.log2(r))) - 7))
    return out


RIDGE_OPS_PER_BYTE = PEAK_INT8_TOPS * 1e12 / (PEAK_HBM_GBS * 1e9)  # ~629 int8 op per HBM byte


def roof_labels(ops, alg_bytes, mfma_frac, hbm_frac):
    """(bound, limiter) of a probed launch.  bound: the roof its arithmetic intensity puts it under
    (algorithmic ops / algorithmic bytes against the ridge point) -- the roof `frac` is priced
    against.  limiter: what the two measured fractions say holds it back -- "mfma" or "hbm" when
    that fraction reaches 0.5, else "latency/issue" (neither roof is close: launch ramp, barriers,
    instruction issue)."""
    bound = "mfma" if ops / max(alg_bytes, 1) >= RIDGE_OPS_PER_BYTE else "hbm"
    fr = {"mfma": mfma_frac or 0.0, "hbm": hbm_frac or 0.0}
    top = max(fr, key=fr.get)
    return bound, (top if fr[top] >= 0.5 else "latency/issue")


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(arch, sample, threads_list, in_hw=0):
    """The oracle's reference-structured restatement of the WHOLE NITIInt8Train step (input
    quantiser, NITI_Conv_Int8 forwards in MNN C4 with the 16x4 GEMM unit and float32
    accumulation, relu / maxpool, NITI_LOSS_Grad, the grad graph's weight and input gradients,
    pool / relu gradients, NITI_SGD) on `sample` images, timed on this host once per thread count
    (batch-split pthreads as NITI_Conv_Int8.cpp:224-229).  Test infrastructure, never the product."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import niti_model_ref as R
    import niti_oracle as O
    layers = {"vgg11": R.vgg11_layers, "lenet": R.lenet_layers,
              "vgg16": lambda: R.vgg16_layers(in_hw or 224)}[arch]()
    classes = 1000 if arch == "vgg16" else 10
    W, S = R.init_weights(layers, seed=17)
    rng = np.random.default_rng(1)
    l0 = layers[0]
    img = rng.integers(0, 256, (sample, l0["ci"], l0["h"], l0["h"])).astype(np.uint8)
    labels = rng.integers(0, classes, sample).astype(np.int32)
    legs = []
    for t in threads_list:
        O.set_threads(t)
        t0 = time.perf_counter()
        x, a = O.quantize_images(img)
        R.train_step(layers, W, S, x, a, labels, classes=classes, impl="mnn", threads=t, acc_mode=O.ACC_F32_SEQ)
        secs = time.perf_counter() - t0
        legs.append({"threads": t, "value": round(sample / secs, 3), "seconds": round(secs, 2)})
    return legs


def cpu_baseline_resnet18(sample, threads_list, hw):
    """The oracle's exact C restatement of the whole ResNet-18 step (oracle/niti_resnet_ref.py:
    input quantiser, convs with the shift rule, relu / max pool, the residual rules, sum pool, loss
    gradient, weight and input gradients, NITI_SGD) on `sample` images, once per thread count.
    Test infrastructure, never the product."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import niti_oracle as O
    import niti_resnet_ref as RR
    convs = RR.resnet18_convs(hw, 1000)
    W, S = RR.init_weights(convs, seed=17)
    crng = np.random.default_rng(1)
    cimg = crng.integers(0, 256, (sample, 3, hw, hw)).astype(np.uint8)
    clab = crng.integers(0, 1000, sample).astype(np.int32)
    legs = []
    for t in threads_list:
        O.set_threads(t)
        t0 = time.perf_counter()
        x, a = O.quantize_images(cimg)
        RR.train_step(convs, W, S, x, a, clab, classes=1000)
        secs = time.perf_counter() - t0
        legs.append({"threads": t, "value": round(sample / secs, 3), "seconds": round(secs, 2)})
    return legs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (GPUs of this node); N > 1 outside torchrun "
                                                           "launches the N ranks itself (default: 1, or WORLD_SIZE)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=0, help="images per GPU per step (0: 256 VGG-11 / LeNet, "
                                                         "64 VGG-16 = BASELINE cfg 4's 512 over 8 GPUs)")
    ap.add_argument("--global-batch", type=int, default=0, help="hold the global batch fixed (strong scaling): "
                                                                "global-batch / N images per GPU")
    ap.add_argument("--spawn-check", action="store_true", help="CPU check of the multi-rank launch (gloo, no GPU)")
    ap.add_argument("--arch", default="vgg11", choices=["vgg11", "lenet", "vgg16", "resnet18"])
    ap.add_argument("--in-hw", type=int, default=0, help="input resolution (0: the architecture's own)")
    ap.add_argument("--cpu-sample", type=int, default=-1, help="images in the CPU baseline sample "
                                                               "(-1: 128 VGG-11, 512 LeNet, 0 VGG-16 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=4, help="first CPU leg (reference default: MnistUtils.cpp:43); "
                                                               "the second leg uses every core of this process")
    ap.add_argument("--int8-input", action="store_true", help="feed pre-quantised int8 x with a fixed exponent "
                                                              "instead of uint8 images through the device quantiser")
    ap.add_argument("--probe-layer", type=int, default=-1, help="layer whose GEMM is timed for the roofline (default: "
                                                                "3, VGG-11 / VGG-16 conv4; LeNet: 1, its 5x5 conv2)")
    ap.add_argument("--probe-phase", type=int, default=-1, help="0 fwd, 1 input grad, 2 weight grad (-1: 2, ResNet-18 0)")
    ap.add_argument("--graph", action="store_true", help="replay the step as a hipGraph")
    ap.add_argument("--no-autotune", action="store_true", help="keep the fixed default GEMM plans")
    ap.add_argument("--overlap", action="store_true",
                    help="weight gradients on a second stream beside the input-gradient chain (measured within 1 %% "
                         "of the single-stream step on MI355X, and it slows the overlapped kernels by sharing the CUs)")
    ap.add_argument("--no-overlap", action="store_true", help="(default) weight gradients on the step stream")
    ap.add_argument("--probe-every", type=int, default=1,
                    help="time the probed launch in one timed step of every K (its begin / end events hold the "
                         "dispatches either side of it back; 0: in none, an A/B diagnostic)")
    ap.add_argument("--probe-plan", default="", help="bm,bn,splits,strategy forced on the probed GEMM after "
                                                     "autotuning (PMC passes re-use the timed run's plan)")
    ap.add_argument("--dp-path", action="store_true", help="diagnostic: run the data-parallel step on one GPU (a "
                                                           "one-rank in-process group: the two-launch row kernels, "
                                                           "the range / gradient collectives as no-ops) to time the "
                                                           "protocol's own cost without the network")
    ap.add_argument("--save-plans", default="", help="write the autotuned GEMM plans to this JSON file")
    ap.add_argument("--load-plans", default="", help="use the GEMM plans of this JSON file (no autotuning): the "
                                                     "profiled and PMC passes replay the timed run's launch sequence")
    ap.add_argument("--wgrad-p16", type=int, default=-1, help="force the P16 weight gradient on every layer it "
                                                              "takes with this many K splits (0: its default; "
                                                              "-1: the autotuner's choice)")
    ap.add_argument("--rc-spec", type=int, default=0, choices=[0, 1, 2],
                    help="fused row kernels' speculative epilogue: 0 off (default), 1 on, 2 always redone "
                         "(results identical; A/B diagnostics)")
    args = ap.parse_args()
    if args.gpus is not None and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus, sys.argv[1:])
    if args.spawn_check:
        return spawn_check(args)
    import numpy as np
    import torch

    world, rank, local = resolve_world(args)
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")  # control plane only; the data path is RCCL in C++

    import niti_amd
    niti_amd._lib.lib().niti_diag_rowconv_speculate(args.rc_spec)
    from niti_amd.model import NitiModel

    arch = {"vgg11": niti_amd.ARCH_VGG11, "lenet": niti_amd.ARCH_LENET, "vgg16": niti_amd.ARCH_VGG16,
            "resnet18": niti_amd.ARCH_RESNET18}[args.arch]
    imagenet = arch in (niti_amd.ARCH_VGG16, niti_amd.ARCH_RESNET18)
    args.batch, scaling = per_gpu_batch(args, world, {niti_amd.ARCH_VGG16: 64, niti_amd.ARCH_RESNET18: 128}.get(arch, 256))
    if args.cpu_sample < 0:
        args.cpu_sample = {niti_amd.ARCH_VGG16: 2, niti_amd.ARCH_LENET: 512, niti_amd.ARCH_RESNET18: 1}.get(arch, 128)
    if args.probe_phase < 0:  # ResNet-18: layer1.0.a's forward (a row-segment conv); the others: conv4's wgrad
        args.probe_phase = 0 if arch == niti_amd.ARCH_RESNET18 else 2
    model = NitiModel(arch, args.batch, args.in_hw)
    model.set_graph(args.graph)
    # (data parallel keeps the default too: a third stream beside the step stream and the gradient
    # communicator's stream would share the process's 4 hardware queues with two RCCL
    # communicators, whose spinning kernels must never queue behind one another)
    overlap = args.overlap and not args.no_overlap
    model.set_overlap(overlap)
    model.keep_grads(False)  # no int8 weight-gradient tap: NITI_SGD consumes the gradient in-kernel
    for i, (w, s) in enumerate(synth_weights(model.layers, seed=17)):
        model.set_weight(i, w, s)
    if world > 1:
        uid = [NitiModel.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        model.attach_comm(uid[0], rank, world, exact=True)
    elif args.dp_path:
        from niti_amd.model import LocalGroup
        dp_group = LocalGroup(1)
        model.attach_local(dp_group, 0, exact=True)

    l0 = model.layers[0]
    rng = np.random.default_rng(100 + rank)
    shape = (args.batch, l0["c_in"], l0["h"], l0["w"])
    if args.int8_input:
        x = torch.from_numpy(rng.integers(-127, 128, shape).astype(np.int8)).cuda()
    else:  # uint8 images: the on-device input quantiser is part of every timed step
        x = torch.from_numpy(rng.integers(0, 256, shape).astype(np.uint8)).cuda()
    labels = torch.from_numpy(rng.integers(0, 1000 if imagenet else 10,
                                           args.batch).astype(np.int32)).cuda()

    def step():
        if args.int8_input:
            model.train_step(x, -3, labels)
        else:
            model.train_step_images(x, labels)

    # Setup (untimed): one step to fill the buffers, then per-shape GEMM plan autotuning
    # (niti_model_autotune: candidate tile / split-K plans timed per layer phase).
    tune_s = 0.0
    p16_default = {i: p for (i, ph), p in model.plans().items() if ph == 2 and p[:2] == (16, 16)}
    if args.load_plans:
        step()
        for k, p in json.load(open(args.load_plans)).items():
            layer, phase = (int(v) for v in k.split(","))
            model.set_plan(layer, phase, p)
    elif not args.no_autotune:
        step()
        ta = time.perf_counter()
        model.autotune()
        torch.cuda.synchronize()
        tune_s = time.perf_counter() - ta
    for i, p in p16_default.items():
        if args.wgrad_p16 >= 0:
            sp = args.wgrad_p16 or p[2]
            model.set_plan(i, 2, (16, 16, sp, 2 if sp > 1 else 0))
    if args.probe_layer < 0:
        args.probe_layer = 1 if arch in (niti_amd.ARCH_LENET, niti_amd.ARCH_RESNET18) else 3
    probe_layer = args.probe_layer if args.probe_layer < len(model.layers) else len(model.layers) - 1
    if args.probe_plan:
        model.set_plan(probe_layer, args.probe_phase, [int(v) for v in args.probe_plan.split(",")])
    plans = model.plans()
    if args.save_plans and rank == 0:
        json.dump({f"{l},{p}": list(v) for (l, p), v in plans.items()}, open(args.save_plans, "w"))

    # The probe (HIP events around one GEMM, on the stream it runs on) is armed before the
    # warmup: the step is replayed as a hipGraph and arming it re-captures the graph, which
    # must not happen inside the timed region.  Warmup launches are read and discarded.
    model.set_probe(probe_layer, args.probe_phase, args.steps + args.warmup)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    model.probe_read()
    model.probe_read_span()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if args.probe_every != 1:
            model.probe_pause(args.probe_every <= 0 or i % args.probe_every != args.probe_every - 1)
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # a fused row-kernel launch whose grid barrier timed out computed garbage: no number from it
    if model.rowconv_error() != 0:
        raise RuntimeError("a fused row-kernel grid barrier timed out in the timed region: results invalid")
    # the speculative pairs (the row kernels' two-launch form and the GEMM path's plan strategy 3):
    # launches B redid, and pairs the row kernels ran in store mode or the GEMM pair settled from an
    # alternate, per layer over warmup + timed steps (fwd redone, fwd stored/alt, dgrad redone, dgrad
    # stored/alt)
    model.probe_pause(False)
    spec = [(s[1], s[2], s[4], s[5]) for s in model.spec_stats()]
    spec = {"redone": sum(a + c for a, _, c, _ in spec), "stored_or_alternate": sum(b + d for _, b, _, d in spec),
            "per_layer": [list(v) for v in spec if any(v)]}
    probe_ms, probe_n = model.probe_read()
    span_ms, span_n = model.probe_read_span()
    # the same launch alone (after the timed region, nothing else on the GPU): in the step the
    # weight gradients share the chip with the input-gradient chain on the other stream
    iso_reps = 20
    model.set_probe(probe_layer, args.probe_phase, iso_reps)
    for _ in range(iso_reps):
        model.run_phase(probe_layer, args.probe_phase)
    torch.cuda.synchronize()
    if model.rowconv_error() != 0:
        raise RuntimeError("a fused row-kernel grid barrier timed out in the isolated re-runs: results invalid")
    iso_ms, iso_n = model.probe_read()
    iso_span_ms, iso_span_n = model.probe_read_span()
    model.set_probe(-1, 0, 0)
    # HIP events on the launch stream time the launch (dispatch to completion, as rocprofv3 does);
    # the weight-gradient kernel also times itself from inside (first block start -> last block
    # end on the device wall clock), which leaves out its launch ramp and end-of-kernel writeback
    span_us = span_ms / span_n * 1e3 if span_n else None
    iso_span_us = iso_span_ms / iso_span_n * 1e3 if iso_span_n else None

    ms_per_step = elapsed / args.steps * 1e3
    images = args.batch * world * args.steps
    value = images / elapsed
    step_ops = 2 * model.step_macs() * world
    tops = step_ops * args.steps / elapsed / 1e12

    pl = model.layers[probe_layer]
    k_ops = 2 * args.batch * pl["oh"] * pl["ow"] * pl["c_out"] * pl["c_in"] * pl["kh"] * pl["kw"]
    k_avg_s = probe_ms / max(probe_n, 1) / 1e3
    achieved = k_ops / k_avg_s / 1e12 if probe_n else None
    iso_s = iso_ms / max(iso_n, 1) / 1e3
    iso_achieved = k_ops / iso_s / 1e12 if iso_n else None
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tfile):
        try:
            tr = json.load(open(tfile))
            key = f"{args.arch}_b{args.batch}_L{probe_layer}_p{args.probe_phase}"
            ent = tr.get(key, {})
            # PMC bytes are per plan: report them only when this run's probed plan is the one the
            # counters were collected under (profiles/traffic.json "plan")
            if list(ent.get("plan", [])) == list(plans[(probe_layer, args.probe_phase)]):
                traffic = ent.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    # the probed launch's HBM fraction (PMC traffic when counted, else the algorithmic bytes: x + dy /
    # w + the int8 output -- forward: x + w + y; weight gradient: x + dy + dw, the same three sizes);
    # its roof by arithmetic intensity and what limits it (roof_labels)
    alg_bytes = args.batch * (pl["h"] * pl["w"] * pl["c_in"] + pl["oh"] * pl["ow"] * pl["c_out"]) + \
        pl["c_out"] * pl["c_in"] * pl["kh"] * pl["kw"]
    hbm_bytes = traffic if traffic else alg_bytes
    mfma_frac = achieved / PEAK_INT8_TOPS if achieved else None
    hbm_frac = hbm_bytes / k_avg_s / (PEAK_HBM_GBS * 1e9) if probe_n else None
    bound, limiter = roof_labels(k_ops, alg_bytes, mfma_frac, hbm_frac)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0 and args.arch == "resnet18":
        all_cores = len(os.sched_getaffinity(0))
        if os.environ.get("OMP_NUM_THREADS", "").isdigit():
            all_cores = max(1, min(all_cores, int(os.environ["OMP_NUM_THREADS"])))
        hw = args.in_hw or 224
        legs = cpu_baseline_resnet18(args.cpu_sample, sorted({args.cpu_threads, all_cores}), hw)
        best = max(legs, key=lambda l: l["value"])
        cpu = {"value": best["value"], "unit": "images/s", "cores": best["threads"], "kind": "port",
               "sample": f"{args.cpu_sample} image(s) at {hw}x{hw} through the whole ResNet-18 step in the oracle's exact "
                         f"C restatement (oracle/niti_resnet_ref.py; conv threads split the batch/channels)",
               "legs": legs, "cpu_model": cpu_model()}
    if rank == 0 and world == 1 and args.cpu_sample > 0 and args.arch in ("vgg11", "lenet", "vgg16"):
        # every core this process may use: the affinity set, capped by the box's CPU share
        # (OMP_NUM_THREADS, 16 per GPU on the pool) -- the thread count is reported as `cores`
        all_cores = len(os.sched_getaffinity(0))
        if os.environ.get("OMP_NUM_THREADS", "").isdigit():
            all_cores = max(1, min(all_cores, int(os.environ["OMP_NUM_THREADS"])))
        legs = cpu_baseline(args.arch, args.cpu_sample, sorted({args.cpu_threads, all_cores}), args.in_hw)
        best = max(legs, key=lambda l: l["value"])
        cpu = {"value": best["value"], "unit": "images/s", "cores": best["threads"], "kind": "port",
               "sample": f"{args.cpu_sample} images through the whole {args.arch.upper()} NITIInt8Train step (input "
                         f"quantiser, fwd + relu/pool, loss grad, weight + input grads, pool/relu grads, NITI_SGD) in the "
                         f"oracle's reference-structured C restatement (MNN C4, 16x4 unit, float32 accumulation)",
               "legs": legs, "cpu_model": cpu_model()}

    phase_name = {0: "forward conv", 1: "input-gradient conv", 2: "weight-gradient conv"}[args.probe_phase]
    pplan = plans[(probe_layer, args.probe_phase)]
    if args.probe_phase == 2 and pplan[0] == 16:
        kname = ("wgrad_p16_kernel: P16 pixel-block operands loaded straight into the MFMA fragments, taps as "
                 f"dy row shifts and x row selection, {pplan[2]} K split(s)"
                 + ("; the slabs summed in the step's sgd_combine launch, not in this time" if pplan[2] > 1 else ""))
    elif args.probe_phase == 2 and pplan[0] == 32:
        kname = ("wgrad_taps_kernel: tap-sharing weight gradient, one padded input region per 64-pixel step "
                 f"for all 9 taps, {pplan[2]} K splits")
    elif args.probe_phase == 2:
        kname = f"gemm_kernel {pplan[0]}x{pplan[1]}, K-major over pixels, {pplan[2]} K splits"
    elif arch == niti_amd.ARCH_RESNET18 and model.layers[probe_layer]["kh"] == 3 and model.layers[probe_layer]["stride"] == 1:
        kname = ("rowconv_fwd_kernel, row-segment register-fed conv with the rescale fused: the speculative pair "
                 "(launch A multiplies and requantises with the layer's previous bit width, launch B exits at once "
                 "while it holds), both launches in the time")
    else:
        kname = f"gemm_kernel {pplan[0]}x{pplan[1]}, implicit im2col"
    line = {
        "metric": METRIC if arch == niti_amd.ARCH_VGG11 else METRIC.replace("VGG-11 batch 256",
                                                                              f"{args.arch.upper()} batch {args.batch}"),
        "value": round(value, 2),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "int8",
        "data": ("synthetic (random int8 x, fixed exponent" if args.int8_input else
                 "synthetic (random uint8 images through the on-device input quantiser") +
                "; random labels; seeded niti_normal_int8 weights)",
        "config": {"workload": (f"{args.arch.upper()} NITI int8 training step (fwd+relu+pool, loss grad, "
                                f"weight grad, input grad, SGD), {l0['c_in']}x{l0['h']}x{l0['w']}"
                                + (", 4096-4096-1000 head" if arch == niti_amd.ARCH_VGG16 else "")
                                if arch not in (niti_amd.ARCH_LENET, niti_amd.ARCH_RESNET18) else
                                "LeNet NITI int8 training step, 1x28x28" if arch == niti_amd.ARCH_LENET else
                                f"ResNet-18 NITI int8 training step (C++ step driver: convs, residual sums, sum pool, "
                                f"1000-class loss grad, weight + input grads, SGD), 3x{l0['h']}x{l0['w']}"),
                   "global_batch": args.batch * world, "per_gpu_batch": args.batch,
                   "parallelism": parallelism_label(world, "RCCL all-reduce MAX ranges + SUM int32 grads"),
                   "streams": "weight gradients beside the input-gradient chain on a second stream" if overlap
                   else "one stream (weight gradient, then input gradient, per layer)"},
        "int8_mfma_tops": round(tops, 2),
        "int8_mfma_frac_of_peak": round(tops / PEAK_INT8_TOPS, 4),
        "roofline": {
            "kernel": f"{args.arch.upper()} conv{probe_layer + 1} {phase_name} launch ({kname}; layer index {probe_layer})",
            "bound": bound,
            "limiter": limiter,
            "hbm_frac": round(hbm_frac, 4) if hbm_frac is not None else None,
            "hbm_bytes_basis": "pmc traffic" if traffic else "algorithmic",
            "achieved": round(achieved, 2) if achieved else None,
            "peak": round(PEAK_INT8_TOPS, 1),
            "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_INT8_TOPS, 4) if achieved else None,
            "traffic": traffic,
            "avg_launch_us": round(k_avg_s * 1e6, 2) if probe_n else None,
            "timing": "HIP events on the launch stream",
            "in_kernel_span_us": round(span_us, 2) if span_us else None,
            "launches": probe_n,
            "ops_per_launch": k_ops,
            "plan": dict(zip(("bm", "bn", "splits", "strategy"), plans[(probe_layer, args.probe_phase)])),
            "isolated": {"avg_launch_us": round(iso_s * 1e6, 2) if iso_n else None,
                         "achieved": round(iso_achieved, 2) if iso_achieved else None,
                         "frac": round(iso_achieved / PEAK_INT8_TOPS, 4) if iso_achieved else None,
                         "launches": iso_n,
                         "in_kernel_span_us": round(iso_span_us, 2) if iso_span_us else None,
                         "note": "same launch re-run alone after the timed region (no side-stream overlap)"},
        },
        "autotune_s": round(tune_s, 2) if not (args.no_autotune or args.load_plans) else None,
        "rowconv_spec": spec,
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)

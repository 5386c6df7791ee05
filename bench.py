"""Throughput of the ResUNet unified training step on MI355X.

Workload (BASELINE.json metric "images/sec ResUNet fwd+bwd (64x64 GTSRB
batch)"; config 3 = 14_train_unified_advanced.py unified step, batch 512,
bf16): one step = the dynamic distortion of a clean 64x64x3 uint8 batch
(14:31-64, draws and pixels on device) + ToTensor of both images
(14:199-202), ResUNet forward, loss = L1 + 0.1 * VGG16-features[:16]
perceptual (14:238-242), full backward, AdamW(lr 2e-4, wd 1e-4) (14:222,
245).  Synthetic GTSRB-shaped clean images generated on device.  --repeats
windows of --steps timed steps each; the median window is reported (SURVEY
§8d: 10 warm-up + 50 timed steps, median of 3).
With --gpus N every rank runs the same per-GPU batch and gradients are
all-reduced over RCCL (weak scaling).  Launched by torch.distributed.run
(WORLD_SIZE set) it is one rank; run directly (``python bench.py --gpus 8``)
it starts the N ranks itself through torch.distributed.run and exits with
their status; a WORLD_SIZE that disagrees with --gpus is an error.

Prints ONE JSON line on rank 0 with the driver's fields plus
  roofline     -- the dominant kernel's algorithmic FLOP rate vs the MFMA peak,
                  timed with HIP events on the launch stream over eager steps
                  run right after the timed windows;
  cpu_baseline -- the CPU restatement of the same step (oracle/, the
                  reference's ATen CPU kernels) on the host cores, bounded
                  sample.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.join(REPO, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd")
for _p in (PKG_ROOT, REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "images/sec ResUNet fwd+bwd (64x64 GTSRB batch) at 1/2/4/8 MI355X; PSNR parity"
# hook-counted conv/convT/linear FLOP per image
FLOP_RESUNET_FWDBWD = 13_698_072_576
FLOP_STEP_WITH_PERC = 18_270_388_224
PEAK = {"bf16": 2516.6, "f32": 157.3}          # dense MFMA TFLOP/s (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0                           # HBM3E (MI355X_MICROARCH.md)
# back-to-back v_mfma_f32_16x16x32_bf16 on random operands, every CU, 2 waves
# per SIMD: the clock the chip holds under MFMA load caps what any kernel can
# reach (tools/mfma_ceiling.hip, profiles/r2a_mfma_ceiling.jsonl)
MFMA_CEILING = 1995.9


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--repeats", type=int, default=3,
                    help="timed windows of --steps steps each; the median window is reported")
    ap.add_argument("--batch", type=int, default=512, help="per-GPU batch")
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-perceptual", action="store_true")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe", action="store_true")
    ap.add_argument("--graph", type=int, default=-1,
                    help="capture the step in a HIP graph and replay it (1/0; default: on)")
    ap.add_argument("--probe-steps", type=int, default=3,
                    help="eager steps timed per kernel for the roofline in graph mode")
    return ap.parse_args()


def algorithmic_bytes(tag):
    """Minimal HBM bytes of one conv GEMM launch from its shape tag
    ("fwd m<mode> NxHxW c<c1>+<c2>-><cout>" / "wgrad m<mode> ..."): every
    activation operand read once and the output written once, bf16 (weights
    and epilogue side operands -- accumulate / mask / BN inputs -- not
    counted, so the achieved rate is a lower bound)."""
    import re
    m = re.match(r"(\w+) m(\d) (\d+)x(\d+)x(\d+) c(\d+)\+(\d+)->(\d+)", tag or "")
    if not m:
        return None
    kind, mode, n, h, w, c1, c2, co = m.group(1), *map(int, m.groups()[1:])
    P = n * h * w
    if kind == "wgrad":
        return 2 * P * (c1 + c2 + (co if mode != 2 else 4 * co))
    if mode == 3:                       # convT down: input on the (2h, 2w) grid
        return 2 * (4 * P * (c1 + c2) + P * co)
    return 2 * P * (c1 + c2 + co)       # conv3x3 / 1x1; convT up: 4 taps x co/4


class KernelProbe:
    """HIP-event timing of every igemm / wgrad launch, per kernel symbol:
    launches, algorithmic FLOP, algorithmic bytes, ms."""

    def __init__(self):
        self.rec = []

    def __call__(self, sym, flops, launch, tag=None):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        launch()
        e.record()
        self.rec.append((sym, flops, s, e, tag))

    def summary(self):
        torch.cuda.synchronize()
        agg = {}
        for sym, fl, s, e, tag in self.rec:
            ms = s.elapsed_time(e)
            a = agg.setdefault(sym, [0, 0.0, 0.0, 0.0])
            a[0] += 1
            a[1] += fl
            a[2] += ms
            a[3] += algorithmic_bytes(tag) or 0.0
        return agg


def _latest_pmc():
    import glob
    import re

    def order(f):
        # run tags are r<round><letters>: r4q is newer than r3aq (round first,
        # then a, ..., z, aa, ...)
        m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(f))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")
    c = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_traffic.json")), key=order)
    return c[-1] if c else None


PMC_TRAFFIC = _latest_pmc()


def _norm_sym(sym):
    return (sym.replace(" ", "").replace("::", "").replace("bf16_t", "bf16").replace("mode", "")
            .rstrip(">"))


def pmc_traffic(sym):
    """HBM bytes per launch of ``sym`` from the committed rocprofv3 PMC
    summary (FETCH_SIZE x2 + WRITE_SIZE, separate passes; tools/pmc_traffic.py):
    the launch-weighted average over every template variant the probe counts
    under ``sym`` (the same launches as ``algorithmic_bytes_per_launch``),
    plus the per-variant table.  Returns (bytes or None, {variant: bytes})."""
    try:
        tab = json.load(open(PMC_TRAFFIC))
    except (OSError, ValueError, TypeError):
        return None, {}
    key = _norm_sym(sym)
    per, tot, n = {}, 0.0, 0
    for k, v in tab.items():
        if _norm_sym(k).startswith(key):
            c = int(v.get("launches_per_pass", 1))
            per[k.lstrip(":")] = {"hbm_bytes_per_launch": v["hbm_bytes_per_launch"],
                                   "launches_per_pass": c}
            tot += v["hbm_bytes_per_launch"] * c
            n += c
    return (round(tot / n) if n else None), per


def cpu_share():
    """CPUs this process may use: the affinity mask, capped by a cgroup v2
    CPU quota (a GPU box grants a share of the host, os.cpu_count() shows all
    of its CPUs)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(math.ceil(int(quota) / int(period)))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(seconds, size):
    """The CPU restatement of the same unified step (oracle, fp32), timed on
    the host with every CPU this process may use: a bounded sample of the
    workload (batch 16)."""
    from oracle import reference_cpu as R
    from oracle import seeded as S
    threads = cpu_share()
    torch.set_num_threads(threads)
    B = 16
    sd = S.model_state_dict("resunet")
    p = {k: v.clone().requires_grad_(v.dtype.is_floating_point and "running" not in k)
         for k, v in sd.items()}
    perc = S.seeded_state_dict(S.load_manifest("perceptual"), seed=5)
    clean = S.image_batch(B, size, size, seed=1)
    bad = S.fog_noise(clean, seed=2)
    names = [k for k, v in p.items() if v.requires_grad]
    st = {}

    def step():
        for k in names:
            p[k].grad = None
        loss = R.unified_loss(R.resunet_forward(p, bad, True), clean, perc)
        loss.backward()
        with torch.no_grad():
            R.adamw_step({k: p[k] for k in names}, {k: p[k].grad for k in names}, st, 2e-4,
                         weight_decay=1e-4)

    step()
    n, t0 = 0, time.perf_counter()
    while True:
        step()
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds and n >= 2:
            break
    return {"value": round(n * B / el, 3), "unit": "images/sec", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
            "sample": f"{n} unified steps (ResUNet fwd+bwd + L1 + 0.1*perceptual + AdamW) at "
                      f"batch {B}, {size}x{size}, fp32, oracle/reference_cpu.py (the reference's "
                      f"ATen CPU kernels) on {threads} threads = this process's CPU share "
                      f"({el:.1f} s); the distortion (DataLoader workers in 14:213) is not in it"}


def launch_plan(gpus, argv, env):
    """How ``bench.py --gpus N`` runs: None = this process is the (only or
    already launched) rank; else the command that starts N rank processes
    (torch.distributed.run, one rank per GPU, rendezvous on 127.0.0.1).
    Raises SystemExit when an outer launcher's WORLD_SIZE disagrees with
    --gpus (a bench line must never claim N GPUs it did not run on)."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus and env.get("RR_BENCH_DP1") != "1":
            raise SystemExit(f"bench: WORLD_SIZE={ws} but --gpus {gpus}")
        return None
    if gpus <= 1:
        return None
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1",
            "--nproc-per-node", str(gpus), "--master-addr", "127.0.0.1",
            "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def main():
    a = parse()
    # --gpus N without an outer launcher: start the N ranks here, before this
    # process touches the GPU (a child process, never an exec), and exit
    # with the launcher's status
    cmd = launch_plan(a.gpus, sys.argv[1:], os.environ)
    if cmd is not None:
        import subprocess
        raise SystemExit(subprocess.call(cmd))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    # rehearsal switches for the N > 1 path on a 1-GPU box (never set by the
    # driver): RR_BENCH_ONE_DEVICE=1 puts every rank on cuda:0,
    # RR_DIST_BACKEND=gloo replaces RCCL (which refuses two ranks on one GPU)
    if os.environ.get("RR_BENCH_ONE_DEVICE") == "1":
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # RR_BENCH_DP1=1 (with torchrun --nproc-per-node 1): the N > 1 step at
    # world size 1 -- an RCCL group of one rank and DataParallel with
    # force_comm, so every bucket all-reduce runs (and is graph-captured)
    dp1 = os.environ.get("RR_BENCH_DP1") == "1"
    if world > 1 or dp1:
        backend = os.environ.get("RR_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    import roadrestore as rr
    from roadrestore import ops
    from roadrestore.optim import flatten_parameters
    from roadrestore.parallel import DataParallel

    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    torch.manual_seed(0)
    model = rr.ResUNet().to(dev)
    model.compute_dtype = dt
    model.train()
    perc = rr.VGGPerceptualLoss().to(dev)
    perc.compute_dtype = dt
    flatten_parameters(model)
    dp = DataParallel(model, force_comm=dp1) if world > 1 or dp1 else None
    gscale = dp.grad_scale if dp else 1.0
    # the HIP graph needs graph-capturable collectives: RcclComm (any N on
    # GPUs); the gloo rehearsal backend runs eagerly
    use_graph = a.graph == 1 or (a.graph == -1 and (dp is None or dp.rccl is not None))
    opt = rr.AdamW(model.parameters(), lr=2e-4, weight_decay=1e-4, capturable=use_graph)

    # synthetic GTSRB-shaped clean images (uint8 RGB, NHWC as decoded); every
    # step distorts them on device (14:31-64: draws + fog / noise / motion
    # blur, rr_distort_random_u8) and applies ToTensor to both (14:199-202,
    # the resample at 64x64 is the identity) -- the reference's DataLoader
    # work, inside the timed step and inside the HIP graph
    from roadrestore import imgproc
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    B, H = a.batch, a.size
    clean_u8 = torch.randint(0, 256, (B, H, H, 3), generator=g, device=dev, dtype=torch.uint8)
    distort = imgproc.RandomDistortion(dev, seed=1000 + rank)
    to_tensor = imgproc.Compose([imgproc.Resize((H, H)), imgproc.ToTensor()])
    w_perc = 0.0 if a.no_perceptual else 0.1

    # the target's perceptual features F(clean) do not depend on the
    # distortion or the restorer: started on a side stream, they overlap both
    # (the kernel probe turns it off: per-kernel durations are taken without
    # a concurrent kernel sharing the chip)
    prefetch = [w_perc != 0.0 and os.environ.get("RR_PERC_PREFETCH", "1") != "0"]

    # the restorer's weight re-pack (after the previous step's AdamW) forked
    # onto a side stream at the step start, overlapping the distortion +
    # ToTensor instead of sitting in front of the first conv (A/B:
    # RR_WEIGHT_PREFETCH=0)
    wprefetch = os.environ.get("RR_WEIGHT_PREFETCH", "1") != "0"

    def step():
        if wprefetch:
            model.prefetch_weights()
        clean = to_tensor(clean_u8)
        if prefetch[0]:
            clean = perc.prefetch_target(clean)
        bad = to_tensor(distort(clean_u8))
        opt.zero_grad(set_to_none=True)
        out = model(bad)
        loss = rr.unified_loss(out, clean, perc, w_perc, grad_scale=gscale)
        loss.backward()
        opt.step()
        return loss

    for _ in range(a.warmup):
        step()
    graph = None
    if use_graph:
        # one whole training step (data distortion + ToTensor, fwd, L1 +
        # perceptual, bwd, AdamW with the device-side step count, weight
        # re-packs) as a HIP graph; the allocator is warmed on the capture
        # side stream first (torch recipe) (the warmup on the side stream
        # keeps older AccumulateGrad nodes on the default stream; the mismatch
        # is intentional and harmless here)
        setw = getattr(torch.autograd.graph, "set_warn_on_accumulate_grad_stream_mismatch", None)
        if setw is not None:
            setw(False)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                step()
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        # at N > 1 the bucket all-reduces (RCCL, comm side stream forked from
        # the capture stream) are recorded into the graph with the rest
        # thread_local: RCCL's watchdog thread keeps polling the events of the
        # eager warmup collectives while this thread captures
        torch.cuda.synchronize()
        try:
            with torch.cuda.graph(graph, capture_error_mode="thread_local"):
                loss_g = step()
            torch.cuda.synchronize()
        except Exception as e:                      # pragma: no cover - safety net
            if world > 1:
                # never time a silently different (eager) N > 1 step
                raise SystemExit(f"bench: HIP-graph capture of the N={world} step failed "
                                 f"({type(e).__name__}: {e})")
            print(f"bench: HIP-graph capture failed ({type(e).__name__}: {e}); "
                  "timing eager steps", file=sys.stderr, flush=True)
            graph = None
            if dp is not None:
                dp.finish()
            torch.cuda.synchronize()
    # the kernel probe (HIP events around every GEMM launch) never runs inside
    # the timed region: it times separate eager steps afterwards
    probe = None
    ops.PROBE = None
    windows = []
    for _ in range(max(1, a.repeats)):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            if graph is not None:
                graph.replay()
            else:
                loss = step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        windows.append(time.perf_counter() - t0)
    if world > 1:
        t = torch.tensor(windows, device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        windows = t.tolist()
    el = sorted(windows)[len(windows) // 2]          # median window (max over ranks)
    if graph is not None:
        loss = loss_g
    if not a.no_probe:
        # kernel durations for the roofline: the same kernels, timed eagerly
        # (every rank runs these steps: the backward's all-reduces pair up)
        probe = KernelProbe()
        ops.PROBE = probe
        prefetch[0] = False
        for _ in range(a.probe_steps):
            step()
        ops.PROBE = None
    loss_v = float(loss.item())
    if not math.isfinite(loss_v):
        raise RuntimeError(f"non-finite loss {loss_v}")

    roof = None
    kernels = None
    if probe is not None:
        agg = probe.summary()
        # the dominant kernel = the template (family) with the most time: the
        # probe names some families per variant (conv3r_kernel<W,BC,...>)
        fams = {}
        for k, v in agg.items():
            f = fams.setdefault(k.split("<")[0], [0, 0.0, 0.0, 0.0])
            for i in range(4):
                f[i] += v[i]
        sym, (cnt, fl, ms, by) = max(fams.items(), key=lambda kv: kv[1][2])
        variants = {k: {"launches": v[0], "avg_launch_ms": round(v[2] / v[0], 4),
                        "tflops": round(v[1] / (v[2] * 1e-3) / 1e12, 1)}
                    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][2])
                    if k.split("<")[0] == sym}
        tflops = fl / (ms * 1e-3) / 1e12
        gbs = by / (ms * 1e-3) / 1e9
        pk = PEAK["bf16" if dt == torch.bfloat16 else "f32"]
        # the bound by the kernel's algorithmic intensity vs the ridge point
        hbm_bound = by > 0 and fl / by < pk * 1e12 / (HBM_PEAK_GBS * 1e9)
        traffic, traffic_per = pmc_traffic(sym)
        roof = {"bound": "hbm" if hbm_bound else "mfma", "kernel": sym,
                "achieved": round(gbs if hbm_bound else tflops, 2),
                "peak": HBM_PEAK_GBS if hbm_bound else pk,
                "unit": "GB/s" if hbm_bound else "TFLOP/s",
                "frac": round(gbs / HBM_PEAK_GBS if hbm_bound else tflops / pk, 4),
                "traffic": traffic,
                "traffic_note": "HBM bytes per launch, launch-weighted over the kernel's "
                                "variants (traffic_variants): rocprofv3 FETCH_SIZE x2 (gfx950) + "
                                "WRITE_SIZE in separate --pmc passes of this bench "
                                f"({os.path.relpath(PMC_TRAFFIC, REPO)})" if traffic else None,
                "traffic_variants": traffic_per or None,
                "probe_variants": variants,
                "launches": cnt, "avg_launch_ms": round(ms / cnt, 4),
                "flop_per_launch": fl / cnt, "algorithmic_bytes_per_launch": by / cnt,
                "mfma_tflops": round(tflops, 2), "mfma_frac": round(tflops / pk, 4),
                "hbm_gbs": round(gbs, 1),
                "mfma_practical_ceiling_tflops": MFMA_CEILING}
        tot_fl = sum(v[1] for v in agg.values())
        tot_ms = sum(v[2] for v in agg.values())
        kernels = {"conv_gemm_ms_per_step": round(tot_ms / a.probe_steps, 3),
                   "conv_gemm_tflops": round(tot_fl / (tot_ms * 1e-3) / 1e12, 2),
                   "probe": f"{a.probe_steps} eager steps after the timed region"}

    imgs = world * B * a.steps
    value = imgs / el
    rec = {
        "metric": METRIC, "value": round(value, 2), "unit": "images/sec", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "bf16" if dt == torch.bfloat16 else "fp32",
        "data": "synthetic GTSRB-shaped 64x64x3 uint8 clean images; per step dynamic distortion "
                "(14:31-64, draws + pixels on device) + ToTensor; random-init weights",
        "config": {"workload": "cfg3: ResUNet unified train step (dynamic distortion + ToTensor, "
                               "fwd + L1 + 0.1*VGG16[:16] perceptual + bwd + AdamW), "
                               "14_train_unified_advanced.py",
                   "global_batch": world * B, "per_gpu_batch": B,
                   "image": [H, H, 3], "parallelism": f"dp{world}",
                   "hip_graph": graph is not None,
                   "flop_per_image": FLOP_STEP_WITH_PERC if w_perc else FLOP_RESUNET_FWDBWD},
        "achieved_model_tflops": round(value * (FLOP_STEP_WITH_PERC if w_perc else
                                                FLOP_RESUNET_FWDBWD) / 1e12, 2),
        # the north star's step-level quantity (MFMA utilisation
        # of ResUNet fwd+bwd): per-GPU img/s x the metric's FLOP per image
        # (13.698 GFLOP, ResUNet fwd+bwd) / the dense MFMA peak, and the same
        # with the perceptual loss's FLOP (18.270 GFLOP per image) counted;
        # `roofline` stays the dominant kernel's fraction
        "step_mfma_frac": round(value / world * FLOP_RESUNET_FWDBWD / 1e12 / PEAK[
            "bf16" if dt == torch.bfloat16 else "f32"], 4),
        "step_mfma_frac_with_perceptual": round(value / world * (FLOP_STEP_WITH_PERC if w_perc else
                                                                 FLOP_RESUNET_FWDBWD) / 1e12 / PEAK[
            "bf16" if dt == torch.bfloat16 else "f32"], 4),
        "loss": round(loss_v, 6),
        "repeats": len(windows),
        "window_ms_per_step": [round(w / a.steps * 1e3, 3) for w in windows],
        "roofline": roof,
        "kernels": kernels,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        rec["cpu_baseline"] = cpu_baseline(a.cpu_baseline_seconds, H)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if dp is not None:
        dp.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

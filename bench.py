"""Benchmark: restored images/sec @256x256, 100 IR-SDE (posterior) steps, DA-CLIP ViT-B/32.

One "step" = restore one batch per GPU: DaCLIP encode_image(control=True) -> noise_state ->
100-step graph-captured posterior loop -> (N>1) RCCL all-gather of the restored tensors.
Inputs are synthetic (random-init weights of the real architectures, synthetic LQ images)
and resident in HBM before the timed region. Weights are created on rank 0 and broadcast
over RCCL. Usage (driver contract):
    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
Run the first way with N > 1 (no WORLD_SIZE in the environment), bench.py starts the N ranks
itself: one `torch.distributed.run` child on 127.0.0.1, launched before any GPU call, whose
exit code it returns. Under a launcher, WORLD_SIZE must equal --gpus.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "da-clip_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "restored images/sec @256x256, 100 IR-SDE steps; PSNR vs ref; 1/2/4/8 MI355X"
MFMA_PEAK = {"bf16": 2500.0, "fp16": 2500.0, "fp32": 157.3, "fp8": 5000.0}   # dense TFLOP/s (MI355X_MICROARCH.md)
HBM_PEAK = 8000.0                                  # GB/s
# Per-dispatch PMC figures by kernel symbol (tools/pmc_bench.sh + tools/pmc_traffic.py).
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--model", default="universal-ir", choices=["universal-ir", "wild-ir"],
                   help="universal-ir: ViT-B/32 DA-CLIP + UIR UNet (BASELINE configs[1]); wild-ir: "
                        "ViT-L/14 + scale-0.5 UNet (configs[3], default 512^2, 2 images per GPU)")
    p.add_argument("--batch", type=int, default=None, help="images per GPU (8; wild-ir 2)")
    p.add_argument("--res", type=int, default=None, help="resolution (256; wild-ir 512)")
    p.add_argument("--T", type=int, default=100)
    p.add_argument("--dtype", default="fp16", choices=["bf16", "fp16", "fp32", "fp8"],
                   help="fp16 (default) = IEEE half storage on the f16 MFMA, fp32 accumulation: the "
                        "16-bit mode that holds the north-star 1e-3 dB PSNR bar; bf16 = the same kernels "
                        "with bf16 storage (BASELINE configs[1] names bf16; same bytes and MFMA rate, 8x "
                        "coarser rounding, measured -6.5e-3 dB, reported under 'modes'); fp8 = bf16 kernels with "
                        "the 64->64 ResBlock block2 convs and the ViT GEMMs on e4m3 MX operands (BASELINE "
                        "configs[4]); fp32 = parity mode")
    p.add_argument("--modes", default="bf16",
                   help="comma-separated extra dtypes measured after the main line on 1 GPU (throughput "
                        "+ PSNR vs the reference), reported under 'modes'; 'none' to skip")
    p.add_argument("--lines", default="mixed8,wild-ir,fp8,fp16-b16,fp32",
                   help="comma-separated extra configuration lines measured after the main line on 1 GPU "
                        "(one warmup + min(steps, 2) timed restores each), reported under 'lines': mixed8 = "
                        "configs[2]'s per-GPU slice on 8 distinct real LQ photos with per-image dPSNR vs the "
                        "reference run of that batch; wild-ir = "
                        "BASELINE configs[3]'s per-GPU slice (ViT-L/14 + scale-0.5 UNet, 512^2, 2 images), fp8 = "
                        "configs[4]'s per-GPU slice (256^2, 16 images, e4m3 GEMMs), fp16-b16 = the same 16 images in "
                        "fp16 (equal-batch comparison for fp8), fp32 = the parity mode on the main workload; "
                        "'none' to skip")
    p.add_argument("--kernel-id", type=int, default=None,
                   help="time one conv class by eager per-launch HIP events instead (kh*100 + variant, e.g. "
                        "312 = 3x3 interleaved-row v4 tiles, 327 = conv3r); default: the kernel symbol with the "
                        "largest in-graph time, from a stamped replay of the captured loop graph")
    p.add_argument("--eager-events", action="store_true",
                   help="also time the roofline kernel's class by HIP events around each launch of an eager "
                        "replay (secondary figure: that replay has no side-stream branches)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-roofline", action="store_true", help="skip the profiled replays (PMC runs)")
    p.add_argument("--no-psnr", action="store_true", help="skip the PSNR-vs-reference sample")
    p.add_argument("--cpu-steps", type=int, default=5, help="UNet steps in the CPU sample (>= 5)")
    p.add_argument("--dry-run", action="store_true",
                   help="launcher / rank wiring check without a GPU: gloo backend, CPU tensors, one "
                        "shard_inputs -> all-gather -> max-over-ranks timing pass; rank 0 prints the JSON "
                        "line with n_gpus and the ranks it saw (tests/test_bench_dist.py)")
    a = p.parse_args()
    if a.gpus < 1:
        p.error("--gpus must be >= 1")
    wild = a.model == "wild-ir"
    a.batch = a.batch or (2 if wild else 8)
    a.res = a.res or (512 if wild else 256)
    return a


def model_setup(args):
    """(UNet config, UNet ctor kwargs, vision cfg, text cfg) of the benchmarked model."""
    from daclip_amd import arch
    if args.model == "wild-ir":
        return (arch.WILD_IR_UNET, dict(context_dim=768, use_degra_context=False, use_image_context=True,
                                        scale=0.5), arch.VIT_L_14, arch.TEXT_L_14)
    return arch.UNetConfig(), dict(context_dim=512, use_degra_context=True, use_image_context=True), \
        arch.VIT_B_32, arch.TEXT_B_32


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """`bench.py --gpus N` (N > 1) outside a launcher: one process per GPU, started as a
    `torch.distributed.run` child (one node, rendezvous on 127.0.0.1) running this same
    command line. The parent has made no GPU call and never execs; it waits and returns the
    child's exit code (the reference's multi-device path is DataParallel,
    config/daclip-sde/models/denoising_model.py:37-42; here it is process-per-GPU)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "4"))
    return subprocess.call(cmd, env=env)


def setup_dist(args):
    """Rank wiring from the launcher's environment. WORLD_SIZE must equal --gpus; the world
    size reported as n_gpus is the process group's own."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws != args.gpus:
        raise SystemExit(f"bench: WORLD_SIZE={ws} but --gpus {args.gpus}: launch with "
                         f"--nproc-per-node {args.gpus}, or run `bench.py --gpus {args.gpus}` alone")
    import datetime
    # A hung rank fails the run after DAC_DIST_TIMEOUT seconds (default 600) instead of
    # stalling it: the RCCL broadcast / all-gather / barriers all inherit this timeout.
    tmo = datetime.timedelta(seconds=float(os.environ.get("DAC_DIST_TIMEOUT", "600")))
    if args.dry_run:
        if ws > 1:
            dist.init_process_group("gloo", timeout=tmo)
    else:
        torch.cuda.set_device(local)
        if ws > 1:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
    if ws > 1:
        ws, rank = dist.get_world_size(), dist.get_rank()
    return ws, rank, local


def dry_run(args, ws, rank):
    """The rank wiring of a bench run without a GPU (gloo, CPU tensors): this rank's shard of
    the global batch, one all-gather of it (the restored-output gather's collective), the
    max-over-ranks timing. Rank 0 prints the JSON line with n_gpus and the ranks seen."""
    from daclip_amd import shard
    R = 8
    n_glob, lo, lq, _ = shard_inputs(args.batch, R, ws, rank, "cpu")
    tag = torch.full((lq.shape[0], 1), float(rank))

    def step():
        return shard.gather_outputs(tag, n_glob)
    out, el = timed_steps(step, args.warmup, args.steps, ws, "cpu")
    ranks = sorted(set(int(v) for v in out[:, 0].tolist()))
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": ws, "ranks_seen": ranks, "global_batch": n_glob,
                          "shard_first_index": lo, "steps": args.steps, "warmup": args.warmup,
                          "elapsed_s_max_over_ranks": el}), flush=True)
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()


def host_cores():
    """CPUs this process may actually run on: the affinity mask, capped by a cgroup v2 CPU
    quota when one is set (a GPU box shows the whole machine in os.cpu_count())."""
    n = len(os.sched_getaffinity(0))
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) / int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(args, sd_unet, sd_clip):
    """Oracle (numpy fp32 restatement of the reference path) on all host cores available to
    this process: DaCLIP encode of one 224^2 image + `cpu_steps` (>= 5) of the 100
    UNet+posterior steps at 256^2, B=1; per-image time = encode + 100 x mean step time
    (SURVEY.md §8d allows timing T=5 and scaling linearly)."""
    from threadpoolctl import threadpool_limits
    from oracle import clip as OC, sde as OS, unet as OU
    from daclip_amd import synth
    cores = host_cores()
    with threadpool_limits(limits=cores):
        img = synth.synth_noise((1, 3, 224, 224), seed=3, tag="cpu_img")
        lq = synth.synth_images(1, args.res, args.res, seed=4)
        t0 = time.perf_counter()
        ic, dc = OC.encode_image(sd_clip, img)
        t_enc = time.perf_counter() - t0
        s = OS.IRSDE(50, args.T, "cosine", 0.005)
        s.mu = lq
        x = s.noise_state(lq, synth.synth_noise(lq.shape, seed=5, tag="cpu_n"))
        t0 = time.perf_counter()
        for i in range(args.cpu_steps):
            t = args.T - i
            eps = OU.forward(sd_unet, x, lq, float(t), dc, ic)
            x = s.posterior_step(x, eps, t, synth.synth_noise(lq.shape, seed=6 + i, tag="cpu_z"))
        t_step = (time.perf_counter() - t0) / args.cpu_steps
    per_img = t_enc + args.T * t_step
    return {"value": 1.0 / per_img, "unit": "images/s", "cores": cores, "kind": "port",
            "host_cpus_visible": os.cpu_count(),
            "sample": f"B=1 {args.res}x{args.res}: 1 DaCLIP encode ({t_enc:.2f}s) + {args.cpu_steps} "
                      f"of {args.T} UNet+posterior steps ({t_step:.2f}s each), numpy fp32 oracle; "
                      f"per-image time = encode + {args.T} x step"}


def psnr_vs_reference(args, clip, dev):
    """PSNR parity of the benchmarked mode against the REFERENCE CPU path on a real restoration:
    tests/golden/restore_rain_256_t100.npz is the reference's predict.py flow run in the
    fixture builder on the 256x256 centre crop of images/3_rain.png (BASELINE configs[0]) with
    the tracking UNet weights of synth.tracking_state_dict (the reference's loop converges,
    98.5 % of its output in (0,1), 27.1 dB vs the LQ) and injected noise. It is restored here
    by this run's encoder handle and a UNet handle of the benchmarked dtype loaded with those
    weights (B=1, 256^2, T=100). delta_db = PSNR(ours, LQ) - PSNR(reference, LQ) on uint8
    (no GT exists for the image); north-star bar |delta_db| < 1e-3."""
    from daclip_amd import arch, synth
    from daclip_amd.unet import ConditionalUNet
    from daclip_amd.sde import IRSDE
    from daclip_amd.preprocess import tensor2img, calculate_psnr
    t0 = time.perf_counter()
    g = np.load(os.path.join(ROOT, "tests", "golden", "restore_rain_256_t100.npz"))
    sd = synth.tracking_state_dict(synth.synth_state_dict(arch.unet_state_spec(arch.UNetConfig()), 0),
                                   g["w_g1"], g["w_g2"], float(g["k"]))
    u = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, device=dev, dtype=args.dtype)
    u.load_state_dict(sd)
    lq = torch.tensor(g["rgb_u8"] / 255.0, dtype=torch.float32).permute(2, 0, 1).unsqueeze(0).to(dev)
    ns = torch.from_numpy(synth.synth_noise(tuple(lq.shape), seed=91, tag="rs_noise_state")).to(dev)
    zs = torch.from_numpy(synth.synth_noise((100,) + tuple(lq.shape), seed=92, tag="rs_steps")).to(dev)
    ic, dc = clip.encode_image(torch.from_numpy(g["img4clip"]).to(dev), control=True)
    s = IRSDE(max_sigma=50, T=100, schedule="cosine", eps=0.005)
    s.set_model(u)
    s.set_mu(lq)
    out = s.reverse_posterior(s.noise_state(lq, noise=ns), noises=zs, text_context=dc, image_context=ic)
    u8 = tensor2img(out[0])
    ref = g["out"][0]
    o = out[0].cpu().numpy()
    inr = (ref > 0) & (ref < 1)
    return {"vs": "reference CPU path (tests/golden/restore_rain_256_t100.npz: predict.py flow on the "
                  "images/3_rain.png 256x256 crop, tracking UNet weights, injected noise)",
            "delta_db": round(float(calculate_psnr(u8, g["lq_u8"]) - calculate_psnr(g["out_u8"], g["lq_u8"])), 6),
            "psnr_vs_reference_u8_db": round(float(calculate_psnr(u8, g["out_u8"])), 3),
            "u8_mismatch": round(float(np.mean(u8 != g["out_u8"])), 5),
            "inrange_max_abs_err": float(np.abs(o - ref)[inr].max()),
            "reference_inrange_frac": round(float(inr.mean()), 4),
            "sample": f"B=1 256x256 T=100 restore in the benchmarked dtype ({time.perf_counter() - t0:.1f}s)"}


def psnr_sample(args, wu_keys, clip, unet_lp, lq, img, dev):
    """Wild-IR (no reference fixture at 512^2): PSNR of the benchmarked 16-bit restore vs the
    fp32 (parity-mode) restore of image 0 at the bench resolution, same contexts and noise."""
    from daclip_amd import synth
    from daclip_amd.unet import ConditionalUNet
    from daclip_amd.sde import IRSDE
    from daclip_amd.preprocess import tensor2img, calculate_psnr
    t0 = time.perf_counter()
    u32 = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], **model_setup(args)[1], device=dev, dtype="fp32")
    u32.load_state_dict(synth.synth_state_dict(wu_keys, 0))
    ic, dc = clip.encode_image(img, control=True)
    R = lq.shape[-1]
    ns = torch.from_numpy(synth.synth_noise((1, 3, R, R), seed=7, tag="psnr_ns")).to(dev)
    zs = torch.from_numpy(synth.synth_noise((args.T, 1, 3, R, R), seed=8, tag="psnr_z")).to(dev)
    outs = {}
    for name, m in ((args.dtype, unet_lp), ("fp32", u32)):
        s = IRSDE(max_sigma=50, T=args.T, schedule="cosine", eps=0.005)
        s.set_model(m)
        s.set_mu(lq)
        x = s.noise_state(lq, noise=ns)
        outs[name] = tensor2img(s.reverse_posterior(x, noises=zs, text_context=dc, image_context=ic)[0])
    gt = tensor2img(lq[0])
    return {f"{args.dtype}_vs_fp32_db": round(float(calculate_psnr(outs[args.dtype], outs["fp32"])), 3),
            "delta_db_on_lq": round(float(calculate_psnr(outs[args.dtype], gt) - calculate_psnr(outs["fp32"], gt)), 5),
            "sample": f"image 0, {R}x{R}, T={args.T}, same contexts + injected noise; fp32 = parity path "
                      f"({time.perf_counter() - t0:.1f}s)"}


def extra_mode(args, dtype, dev, lq, img4clip, uspec, cspec):
    """Another compute dtype on the same workload (1 GPU): its own handles, `warmup` + `steps`
    timed restores of the same batch, and its PSNR against the reference fixture."""
    from daclip_amd import synth
    from daclip_amd.unet import ConditionalUNet
    from daclip_amd.open_clip import DaCLIP
    from daclip_amd.sde import IRSDE
    ucfg, ukw, vcfg, tcfg = model_setup(args)
    unet = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], **ukw, device=dev, dtype=dtype)
    unet.load_state_dict(synth.synth_state_dict(uspec, 0))
    clip = DaCLIP(vcfg, tcfg, device=dev, dtype=dtype, with_text=False)
    clip.load_state_dict(synth.synth_state_dict(cspec, 0), strict=False)
    sde = IRSDE(max_sigma=50, T=args.T, schedule="cosine", eps=0.005)
    sde.set_model(unet)
    sde.set_mu(lq)

    def step():
        ic, dc = clip.encode_image(img4clip, control=True)
        return sde.reverse_posterior(sde.noise_state(lq), text_context=dc, image_context=ic)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    B = lq.shape[0]
    res = {"dtype": dtype, "value": round(B * args.steps / el, 4), "unit": "images/s",
           "ms_per_step": round(el / args.steps * 1e3, 2), "outputs_finite": bool(torch.isfinite(out).all().item())}
    if args.model == "universal-ir" and args.T == 100 and not args.no_psnr:
        a2 = argparse.Namespace(**vars(args))
        a2.dtype = dtype
        res["psnr"] = psnr_vs_reference(a2, clip, dev)
    return res


def shard_inputs(batch, R, ws, rank, dev):
    """Weak scaling: the global batch is ws * batch images and rank r takes its contiguous shard
    (shard.shard_bounds). Inputs are keyed by GLOBAL image index, and so is the device noise
    (sde.image_offset, set by make_step), so every image restores identically for any world
    size. Returns (n_global, first global index, lq [b,3,R,R], img4clip [b,3,224,224])."""
    from daclip_amd import shard, synth
    n_glob = ws * batch
    lo, hi = shard.shard_bounds(n_glob, ws, rank)
    lq = torch.from_numpy(np.concatenate([synth.synth_images(1, R, R, seed=100 + g) for g in range(lo, hi)]
                                         or [np.zeros((0, 3, R, R), np.float32)])).to(dev)
    img4clip = torch.from_numpy(np.concatenate([synth.synth_noise((1, 3, 224, 224), seed=200 + g, tag="clip")
                                                for g in range(lo, hi)] or [np.zeros((0, 3, 224, 224), np.float32)])).to(dev)
    return n_glob, lo, lq, img4clip


def make_step(clip, sde, lq, img4clip, lo, n_glob, ws):
    """One bench step on this rank: encode_image(control=True) -> noise_state -> the T-step
    posterior loop over this rank's shard -> (ws > 1) one all-gather of the restored images."""
    from daclip_amd import shard
    sde.set_mu(lq)
    sde.image_offset = lo

    def step():
        ic, dc = clip.encode_image(img4clip, control=True)
        noisy = sde.noise_state(lq)
        out = sde.reverse_posterior(noisy, text_context=dc, image_context=ic)
        if ws > 1:
            out = shard.gather_outputs(out, n_glob)
        return out
    return step


def _sync(dev):
    if torch.device(dev).type == "cuda":
        torch.cuda.synchronize(dev)


def timed_steps(step, warmup, steps, ws, dev):
    """`warmup` untimed steps, then exactly `steps` timed ones bracketed by a barrier + device
    synchronize on both sides; the elapsed time is the MAX over ranks. Returns (last output, s)."""
    for _ in range(warmup):
        step()
    _sync(dev)
    if ws > 1:
        dist.barrier()
    _sync(dev)
    t0 = time.perf_counter()
    out = None
    for _ in range(steps):
        out = step()
    _sync(dev)
    if ws > 1:
        dist.barrier()
    _sync(dev)
    el = time.perf_counter() - t0
    if ws > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return out, el


def profile_class(h, step, kernel_id):
    """Eager replay of one more restore of the same batch on the same stream with HIP events
    around every launch of conv class `kernel_id` (999 = every conv launch). The eager replay
    records the UNet without its side-stream branches (full-batch launches), so it is a
    secondary figure; the roofline comes from graph_profile. Returns (launches, mean ms per
    launch, FLOPs per launch, algorithmic bytes per launch, eager ms, per-launch rows)."""
    from daclip_amd import _lib
    mean_ms, fl, by = _lib.ctypes.c_double(), _lib.ctypes.c_double(), _lib.ctypes.c_double()
    h.check(_lib.lib().dac_profile_enable(h.h, kernel_id), "profile_enable")
    torch.cuda.synchronize()
    tp = time.perf_counter()
    step()
    torch.cuda.synchronize()
    eager_ms = (time.perf_counter() - tp) * 1e3
    n = _lib.lib().dac_profile_read(h.h, _lib.ctypes.byref(mean_ms), _lib.ctypes.byref(fl), _lib.ctypes.byref(by))
    rows = _launch_rows(h, n)
    h.check(_lib.lib().dac_profile_enable(h.h, -1), "profile_disable")
    return max(n, 0), mean_ms.value, fl.value, by.value, eager_ms, rows


def _launch_rows(h, n):
    """(ms, flops, bytes, class, label, symbol) of each launch of the last profile."""
    from daclip_amd import _lib
    c = _lib.ctypes
    rows = []
    for i in range(max(n, 0)):
        ms, fl, by, cls, t0, br = c.c_double(), c.c_double(), c.c_double(), c.c_int(), c.c_double(), c.c_int()
        lab, sym = c.create_string_buffer(200), c.create_string_buffer(400)
        h.check(_lib.lib().dac_profile_launch(h.h, i, c.byref(ms), c.byref(fl), c.byref(by), c.byref(cls),
                                              c.byref(t0), c.byref(br), lab, 200, sym, 400), "profile_launch")
        rows.append((ms.value, fl.value, by.value, cls.value, lab.value.decode(), sym.value.decode(),
                     t0.value, br.value))
    return rows


def time_shares(rows):
    """Per launch: its in-graph duration divided among the conv launches running at the same
    time (the UNet's split section runs two half-batch branches concurrently): the integral
    over the launch's [start, end] of 1 / (number of profiled launches active). Sums to the
    busy time of the profiled kernels; non-conv kernels of the other branch are not counted."""
    ev = []
    for i, r in enumerate(rows):
        ev.append((r[6], 1, i))
        ev.append((r[6] + r[0], -1, i))
    ev.sort()
    share = [0.0] * len(rows)
    active = set()
    last = None
    for t, d, i in ev:
        if last is not None and active and t > last:
            w = (t - last) / len(active)
            for j in active:
                share[j] += w
        last = t
        if d > 0:
            active.add(i)
        else:
            active.discard(i)
    return share


def graph_profile(h, step):
    """Every conv launch of one restore timed INSIDE a replay of the captured loop graph
    (dac_profile_mode 1): the engine records and captures the loop exactly as the timed graph
    (same kernels, grids, arena and side-stream branches), each launch carrying a wall-clock
    [begin, end] stamp pair it writes itself (HIP events cannot be timed inside graph
    replays), replays it once with HIP events around the replay on the loop's stream, and
    names each launch's kernel symbol from the captured graph's nodes.
    Returns (per-launch rows, graph replay ms by HIP events, host ms of the profiled step)."""
    from daclip_amd import _lib
    L = _lib.lib()
    h.check(L.dac_profile_mode(h.h, 1), "profile_mode")
    try:
        h.check(L.dac_profile_enable(h.h, 999), "profile_enable")
        torch.cuda.synchronize()
        tp = time.perf_counter()
        step()
        torch.cuda.synchronize()
        step_ms = (time.perf_counter() - tp) * 1e3
        n = h.check(L.dac_profile_read(h.h, None, None, None), "profile_read")
        rows = _launch_rows(h, n)
        gms = _lib.ctypes.c_double()
        h.check(L.dac_profile_graph_ms(h.h, _lib.ctypes.byref(gms)), "profile_graph_ms")
    finally:
        L.dac_profile_enable(h.h, -1)
        L.dac_profile_mode(h.h, 0)
    return rows, gms.value, step_ms


def pmc_symbol(sym):
    """Per-dispatch PMC figures of one kernel symbol (profiles/pmc_traffic.json), or None."""
    if not sym or not os.path.exists(PMC_FILE):
        return None
    with open(PMC_FILE) as f:
        ks = json.load(f)["kernels"]
    es = [ks[x] for x in sym.split("+") if x in ks and "hbm_bytes_per_dispatch" in ks[x]]
    if not es:
        return None
    n = sum(e["dispatches"] for e in es)
    out = {"dispatches": n, "hbm_bytes_per_dispatch": sum(e["hbm_bytes_total"] for e in es) / n}
    if all("mfma_busy" in e for e in es):
        out["mfma_busy"] = sum(e["mfma_busy"] * e["dispatches"] for e in es) / n
    return out


def _group(rows, key, shares=None):
    g = {}
    for i, (ms, fl, by, cls, lab, sym, t0, br) in enumerate(rows):
        k = key(cls, sym)
        e = g.setdefault(k, {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0, "classes": set(),
                             "symbols": set(), "branch": 0, "share_ms": 0.0})
        e["launches"] += 1
        e["ms"] += ms
        e["flops"] += fl
        e["bytes"] += by
        e["classes"].add(cls)
        e["symbols"].add(sym)
        e["branch"] += br
        e["share_ms"] += shares[i] if shares else ms
    return g


def dominant_roofline(h, step, dtype, step_ms, pmc_ok=False, eager=True):
    """Roofline of the kernel (symbol) with the largest in-graph time per restore, from one
    stamped replay of the captured loop graph (graph_profile): achieved = its launches'
    algorithmic FLOPs / their summed in-graph durations. Also every symbol's and every conv
    class's share, and (secondary) the eager per-launch HIP-event figure of the same class."""
    rows, graph_ms, prof_step_ms = graph_profile(h, step)
    if not rows:
        return None
    if os.environ.get("BENCH_PROFILE_DUMP"):          # per-launch rows for offline analysis
        with open(os.environ["BENCH_PROFILE_DUMP"], "w") as f:
            json.dump({"graph_ms": graph_ms, "rows": rows}, f)
    peak = MFMA_PEAK[dtype]
    shares = time_shares(rows)
    syms = _group(rows, lambda c, s: s or f"class {c}", shares)
    dom, e = max(syms.items(), key=lambda kv: kv[1]["ms"])
    ach = e["flops"] / (e["ms"] * 1e-3) / 1e12
    pmc = pmc_symbol(dom) if pmc_ok else None
    r = {"kernel": dom, "kernel_classes": sorted(e["classes"]),
         "bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s", "frac": round(ach / peak, 4),
         "traffic": pmc["hbm_bytes_per_dispatch"] if pmc else None,
         "traffic_source": ("profiles/pmc_traffic.json: 2*FETCH_SIZE+WRITE_SIZE (KiB->B, gfx950 x2 read "
                            "correction) per dispatch of this symbol, rocprofv3 --pmc over this bench command")
         if pmc else None,
         "mfma_busy_pmc": round(pmc["mfma_busy"], 4) if pmc and "mfma_busy" in pmc else None,
         "launches_per_restore": e["launches"], "mean_launch_us": round(e["ms"] / e["launches"] * 1e3, 2),
         "flops_per_launch": e["flops"] / e["launches"], "algorithmic_bytes_per_launch": e["bytes"] / e["launches"],
         "achieved_hbm_GBps": round(e["bytes"] / (e["ms"] * 1e-3) / 1e9, 1),
         "ms_per_restore": round(e["ms"], 3),
         "launches_in_concurrent_branches": e["branch"],
         "frac_time_shared": round(e["flops"] / (e["share_ms"] * 1e-3) / 1e12 / peak, 4),
         "frac_time_shared_note": ("FLOPs / the launches' in-graph time divided among the profiled (conv) "
                                   "launches running at the same time (two half-batch branches share the chip "
                                   "in the split section); frac uses the undivided durations"),
         "measured_on": (f"in-graph launch durations: one replay of the captured {len(rows)}-conv-launch loop "
                         f"graph (the timed graph's kernels, grids and side-stream branches) with a wall-clock "
                         f"[begin, end] stamp pair per launch written by the kernel (s_memrealtime, 100 MHz); "
                         f"replay {graph_ms:.1f} ms by HIP events on the loop's stream, profiled step "
                         f"{prof_step_ms:.1f} ms vs timed step {step_ms:.1f} ms"),
         "selection": "kernel symbol with the largest summed in-graph duration per restore"}
    if pmc and "mfma_busy" in pmc:
        r["mfma_busy_note"] = ("PMC MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs) on "
                               "dispatches serialised by counter collection (no branch overlap), at the "
                               "profiled clock; frac = FLOPs / in-graph duration / 2.5 PF at the nominal clock")
    r["symbols"] = [{"symbol": k, "classes": sorted(v["classes"]), "launches": v["launches"],
                     "ms_per_restore": round(v["ms"], 3), "mean_us": round(v["ms"] / v["launches"] * 1e3, 2),
                     "flops_per_launch": v["flops"] / v["launches"],
                     "frac_of_peak": round(v["flops"] / (v["ms"] * 1e-3) / 1e12 / peak, 4),
                     "in_branches": v["branch"],
                     "frac_time_shared": round(v["flops"] / (v["share_ms"] * 1e-3) / 1e12 / peak, 4)}
                    for k, v in sorted(syms.items(), key=lambda kv: -kv[1]["ms"])[:16]]
    cls = _group(rows, lambda c, s: c, shares)
    r["classes"] = [{"class": k, "launches": v["launches"], "ms_per_restore": round(v["ms"], 3),
                     "frac_of_peak": round(v["flops"] / (v["ms"] * 1e-3) / 1e12 / peak, 4)}
                    for k, v in sorted(cls.items(), key=lambda kv: -kv[1]["ms"])]
    r["conv_ms_per_restore_in_graph"] = round(sum(v["ms"] for v in cls.values()), 3)
    r["conv_busy_ms_per_restore"] = round(sum(shares), 3)
    r["conv_tflops_per_restore"] = round(sum(x[1] for x in rows) / 1e12, 3)
    if eager:
        # Secondary: the same class(es) by HIP events around each launch of an eager replay
        # (no side-stream branches there: full-batch launches, so launch counts differ).
        n, _, _, _, eager_ms, erows = profile_class(h, step, 999)
        ecls = _group(erows, lambda c, s: c)
        sel = [v for k, v in ecls.items() if k in e["classes"]]
        if sel:
            ms = sum(v["ms"] for v in sel)
            fl = sum(v["flops"] for v in sel)
            nl = sum(v["launches"] for v in sel)
            r["eager_events"] = {"classes": sorted(e["classes"]), "launches": nl, "mean_launch_us": round(ms / nl * 1e3, 2),
                                 "frac": round(fl / (ms * 1e-3) / 1e12 / peak, 4), "eager_step_ms": round(eager_ms, 1)}
    return r


def roofline_entry(kernel_id, dtype, n, mean_ms, fl, by, eager_ms, graph_ms, pmc=None):
    """--kernel-id: one conv class by the eager per-launch HIP events (secondary method)."""
    ach = fl / (mean_ms * 1e-3) / 1e12
    return {"kernel": f"conv_kernel class {kernel_id} (kh*100 + variant, {dtype})",
            "bound": "mfma", "achieved": round(ach, 2), "peak": MFMA_PEAK[dtype],
            "unit": "TFLOP/s", "frac": round(ach / MFMA_PEAK[dtype], 4),
            "traffic": pmc["hbm_bytes_per_dispatch"] if pmc else None,
            "launches_timed": n, "mean_launch_us": round(mean_ms * 1e3, 2),
            "flops_per_launch": fl, "algorithmic_bytes_per_launch": by,
            "measured_on": f"eager replay of one batch (events per launch), {eager_ms:.1f} ms vs graph "
                           f"{graph_ms:.1f} ms/step"}


LINES = {
    # name: (model, resolution, images per GPU, dtype or None = the main line's, BASELINE config)
    "wild-ir": ("wild-ir", 512, 2, None, "configs[3] per-GPU slice: Wild-IR 512x512, 16 images over 8 GPUs"),
    "fp8": ("universal-ir", 256, 16, "fp8", "configs[4] per-GPU slice: fp8 GEMMs, 256x256, 128 images over 8 GPUs. "
                                           "A coverage / precision line, not a speed path: it measures within "
                                           "+-1 % of fp16 at the same batch (line fp16-b16) with dPSNR +0.06 dB "
                                           "(DESIGN.md §3, fp8)"),
    "fp32": ("universal-ir", 256, 8, "fp32", "configs[1] workload in the fp32 parity mode"),
    "fp16-b16": ("universal-ir", 256, 16, "fp16", "configs[4]'s per-GPU batch (16 images) in fp16: the fp8 "
                                                  "line's equal-batch 16-bit comparison"),
}


def mixed_line(args, dev):
    """BASELINE configs[2]'s per-GPU slice on REAL inputs: the 8 distinct LQ photos of
    tests/golden/mixed8_256_t100.npz (rain, haze, motion blur, low light, ... 256x256 crops of the
    reference's sample images) as one B=8 batch in the benchmarked dtype, with the restoration
    fixture's tracking UNet weights (synth.tracking_state_dict) and seed-0 ViT-B/32. Throughput:
    the same step as the main line (encode -> noise_state -> graph loop, device noise), one warmup
    and min(steps, 2) timed restores. Parity: one more restore with the fixture's injected noise,
    every image's dPSNR against the reference's run of the same batch, and the degradation-class
    argmax (text tower on this GPU) against the reference's."""
    from daclip_amd import arch, synth
    from daclip_amd.unet import ConditionalUNet
    from daclip_amd.open_clip import DaCLIP
    from daclip_amd.sde import IRSDE
    from daclip_amd.preprocess import tensor2img, calculate_psnr
    t0 = time.perf_counter()
    gd = os.path.join(ROOT, "tests", "golden")
    g = np.load(os.path.join(gd, "mixed8_256_t100.npz"))
    r = np.load(os.path.join(gd, "restore_rain_256_t100.npz"))
    sd = synth.tracking_state_dict(synth.synth_state_dict(arch.unet_state_spec(arch.UNetConfig()), 0),
                                   r["w_g1"], r["w_g2"], float(r["k"]))
    unet = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], 512, True, True, device=dev, dtype=args.dtype)
    unet.load_state_dict(sd)
    clip = DaCLIP(arch.VIT_B_32, arch.TEXT_B_32, device=dev, dtype=args.dtype)
    clip.load_synthetic(seed=0)
    sde = IRSDE(max_sigma=50, T=100, schedule="cosine", eps=0.005)
    sde.set_model(unet)
    lq = torch.tensor(g["rgb_u8"] / 255.0, dtype=torch.float32).permute(0, 3, 1, 2).contiguous().to(dev)
    img = torch.from_numpy(g["img4clip"]).to(dev)
    B = lq.shape[0]
    k = min(args.steps, 2)
    out, el = timed_steps(make_step(clip, sde, lq, img, 0, B, 1), 1, k, 1, dev)
    res = {"line": "mixed8", "config": "configs[2] per-GPU slice on real inputs: 8 distinct LQ photos "
                                       "(tests/golden/mixed8_256_t100.npz), 256x256, one batch",
           "images": [str(x) for x in g["names"]], "dtype": args.dtype, "batch_per_gpu": B,
           "value": round(B * k / el, 4), "unit": "images/s", "ms_per_step": round(el / k * 1e3, 2), "steps": k,
           "outputs_finite": bool(torch.isfinite(out).all().item())}
    if not args.no_psnr:
        shape = (B, 3, 256, 256)
        n0 = torch.from_numpy(synth.synth_noise(shape, seed=91, tag="mx_noise_state")).to(dev)
        zs = torch.from_numpy(synth.synth_noise((100,) + shape, seed=92, tag="mx_steps")).to(dev)
        ic, dc = clip.encode_image(img, control=True)
        t = np.load(os.path.join(gd, "text_b32.npz"))
        _, am = clip.degradation_probs(dc, clip.encode_text(torch.from_numpy(t["tokens"])))
        sde.set_mu(lq)
        o = sde.reverse_posterior(sde.noise_state(lq, noise=n0), noises=zs, text_context=dc, image_context=ic)
        o = o.cpu()
        d = [float(calculate_psnr(tensor2img(o[b]), g["lq_u8"][b]) - calculate_psnr(g["out_u8"][b], g["lq_u8"][b]))
             for b in range(B)]
        res["psnr"] = {"vs": "reference CPU path on the same batch (make_golden.py gen_mixed)",
                       "delta_db": [round(x, 6) for x in d], "max_abs_delta_db": round(max(map(abs, d)), 6),
                       "mean_delta_db": round(float(np.mean(d)), 6),
                       "argmax": am.cpu().numpy().tolist(), "argmax_equals_reference":
                           bool(np.array_equal(am.cpu().numpy(), g["argmax"]))}
    res["wall_s"] = round(time.perf_counter() - t0, 1)
    return res


def extra_line(args, name, dev):
    """One more BASELINE configuration on this GPU (driver-observed in the same run): its own
    handles with the seeded synthetic weights, the same step as the main line (encode ->
    noise_state -> T-step graph loop), one warmup and min(steps, 2) timed restores."""
    from daclip_amd import arch, synth
    from daclip_amd.unet import ConditionalUNet
    from daclip_amd.open_clip import DaCLIP
    from daclip_amd.sde import IRSDE
    model, R, B, dt, what = LINES[name]
    a2 = argparse.Namespace(**vars(args))
    a2.model, a2.res, a2.batch, a2.dtype = model, R, B, dt or args.dtype
    t0 = time.perf_counter()
    ucfg, ukw, vcfg, tcfg = model_setup(a2)
    uspec = arch.unet_state_spec(ucfg)
    cspec = {k: s for k, s in arch.daclip_state_spec(vcfg, tcfg).items() if k.startswith(("clip.visual.", "visual_control."))}
    unet = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], **ukw, device=dev, dtype=a2.dtype)
    unet.load_state_dict(synth.synth_state_dict(uspec, 0))
    clip = DaCLIP(vcfg, tcfg, device=dev, dtype=a2.dtype, with_text=False)
    clip.load_state_dict(synth.synth_state_dict(cspec, 0), strict=False)
    sde = IRSDE(max_sigma=50, T=a2.T, schedule="cosine", eps=0.005)
    sde.set_model(unet)
    n, lo, lq, img = shard_inputs(B, R, 1, 0, dev)
    out, el = timed_steps(make_step(clip, sde, lq, img, lo, n, 1), 1, min(args.steps, 2), 1, dev)
    k = min(args.steps, 2)
    ref_tf = arch.reference_tflop_per_image(ucfg, vcfg, R, R, a2.T)
    res = {"line": name, "config": what, "model": model, "dtype": a2.dtype, "resolution": R, "batch_per_gpu": B,
           "value": round(B * k / el, 4), "unit": "images/s", "ms_per_step": round(el / k * 1e3, 2), "steps": k,
           "outputs_finite": bool(torch.isfinite(out).all().item()),
           "model_tflop_per_image": round((a2.T * unet.flops(B, R, R) + clip.flops(B)) / B / 1e12, 3),
           "reference_tflop_per_image": round(ref_tf, 3),
           "whole_path_frac_of_peak": round(ref_tf * B * k / el / MFMA_PEAK[a2.dtype], 4)}
    if model == "universal-ir" and a2.T == 100 and not args.no_psnr:
        res["psnr"] = psnr_vs_reference(a2, clip, dev)
    elif model == "wild-ir" and not args.no_psnr and a2.dtype in ("bf16", "fp16"):
        # No reference fixture exists at 512^2: the 16-bit restore against this line's fp32
        # parity-mode restore of image 0 (same weights, contexts and injected noise).
        res["psnr"] = psnr_sample(a2, arch.unet_state_spec(ucfg), clip, unet, lq[:1], img[:1], dev)
    if model == "wild-ir" and not args.no_roofline:
        step = make_step(clip, sde, lq, img, lo, n, 1)
        res["roofline"] = dominant_roofline(unet._h, step, a2.dtype, el / k * 1e3, eager=False)
    res["wall_s"] = round(time.perf_counter() - t0, 1)
    return res


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    ws, rank, local = setup_dist(args)
    if args.dry_run:
        return dry_run(args, ws, rank)
    dev = torch.device("cuda", local)
    from daclip_amd import arch, synth, _lib, shard
    from daclip_amd.unet import ConditionalUNet
    from daclip_amd.open_clip import DaCLIP
    from daclip_amd.sde import IRSDE

    ucfg, ukw, vcfg, tcfg = model_setup(args)
    uspec = arch.unet_state_spec(ucfg)
    cspec = {k: s for k, s in arch.daclip_state_spec(vcfg, tcfg).items()
             if k.startswith(("clip.visual.", "visual_control."))}
    sd_u = synth.synth_state_dict(uspec, 0) if rank == 0 else None
    sd_c = synth.synth_state_dict(cspec, 0) if rank == 0 else None
    wu = shard.broadcast_state(sd_u, list(uspec), dev)
    wc = shard.broadcast_state(sd_c, list(cspec), dev)

    unet = ConditionalUNet(3, 3, 64, [1, 2, 4, 8], **ukw, device=dev, dtype=args.dtype)
    unet.load_state_dict(wu)
    clip = DaCLIP(vcfg, tcfg, device=dev, dtype=args.dtype, with_text=False)
    clip.load_state_dict(wc, strict=False)
    del wu, wc
    sde = IRSDE(max_sigma=50, T=args.T, schedule="cosine", eps=0.005)
    sde.set_model(unet)

    R = args.res
    n_glob, lo, lq, img4clip = shard_inputs(args.batch, R, ws, rank, dev)
    B = lq.shape[0]
    step = make_step(clip, sde, lq, img4clip, lo, n_glob, ws)
    h = unet._h
    out, el = timed_steps(step, args.warmup, args.steps, ws, dev)

    finite = bool(torch.isfinite(out).all().item())
    if not finite:
        # fp16 storage saturates at 65504: a non-finite restore is an error, never a number.
        raise SystemExit(f"bench: non-finite restored outputs in {args.dtype} mode")
    n_launch, mean_ms, fl, by, eager_ms = 0, 0.0, 0.0, 0.0, 0.0
    roof = None
    # The committed PMC passes were collected on the default workload only.
    default_wl = args.model == "universal-ir" and args.batch == 8 and args.res == 256
    if not args.no_roofline:
        # Roofline of the dominant kernel class (HIP events per launch on the kernel's stream).
        if args.kernel_id is None:
            roof = dominant_roofline(h, step, args.dtype, el / args.steps * 1e3, pmc_ok=default_wl,
                                     eager=args.eager_events)
        else:
            n_launch, mean_ms, fl, by, eager_ms, _ = profile_class(h, step, args.kernel_id)
            if n_launch > 0:
                roof = roofline_entry(args.kernel_id, args.dtype, n_launch, mean_ms, fl, by, eager_ms,
                                      el / args.steps * 1e3)

    psnr = None
    if rank == 0 and not args.no_psnr:
        if args.model == "universal-ir" and args.T == 100:
            psnr = psnr_vs_reference(args, clip, dev)
        elif args.dtype in ("bf16", "fp16"):
            psnr = psnr_sample(args, wu_keys=uspec, clip=clip, unet_lp=unet, lq=lq[:1], img=img4clip[:1], dev=dev)

    if rank == 0:
        images = n_glob * args.steps
        uflops = unet.flops(B, R, R)
        eflops = clip.flops(B)
        total_tf = (args.T * uflops + eflops) / B / 1e12
        ref_tf = arch.reference_tflop_per_image(ucfg, vcfg, R, R, args.T)
        wild = args.model == "wild-ir"
        metric = METRIC if not wild else METRIC.replace("@256x256", f"@{R}x{R} (Wild-IR)")
        res = {"metric": metric, "value": round(images / el, 4), "unit": "images/s", "n_gpus": ws,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 2),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
               "data": ("synthetic (random-init ViT-L/14 DA-CLIP + Wild-IR scale-0.5 ConditionalUNet, synthetic LQ)"
                        if wild else "synthetic (random-init ViT-B/32 DA-CLIP + nf=64 ConditionalUNet, synthetic LQ)"),
               "config": {"workload": (f"Wild-IR synthetic batch, {R}x{R}, batch={B}/GPU, {args.T} IR-SDE "
                                       f"posterior steps, hipGraph loop (BASELINE configs[3])") if wild else
                                      (f"deraining-shaped synthetic batch, {R}x{R}, batch={B}/GPU, "
                                       f"{args.T} IR-SDE posterior steps, hipGraph loop (BASELINE configs[1])"),
                          "model": args.model,
                          "batch_per_gpu": B, "global_batch": n_glob, "resolution": R, "sde_steps": args.T,
                          "sampler": "posterior", "parallelism": f"dp{ws}"},
               # executed work (the engine's count) and the reference-defined work (SURVEY §8(d),
               # arch.reference_tflop_per_image: 26.635 TF per 256^2 image at T = 100)
               "model_tflop_per_image": round(total_tf, 3),
               "reference_tflop_per_image": round(ref_tf, 3),
               "whole_path_tflops": round(total_tf * images / el, 1),
               "whole_path_frac_of_peak": round(ref_tf * images / el / MFMA_PEAK[args.dtype], 4),
               "roofline": roof, "outputs_finite": finite, "psnr": psnr,
               "build": _lib.build_info()}
        modes = [m for m in args.modes.split(",") if m and m != "none" and m != args.dtype]
        if ws == 1 and modes:
            res["modes"] = [extra_mode(args, m, dev, lq, img4clip, uspec, cspec) for m in modes]
            # BASELINE configs[1] names bf16: its number, measured in this run, at the top level
            # so comparisons against the baseline config are made in its own dtype.
            for m in res["modes"]:
                if m["dtype"] == "bf16" and args.model == "universal-ir" and args.batch == 8 and R == 256:
                    res["baseline_config_value"] = {
                        "config": "BASELINE configs[1]: 256x256, batch=8, 100 steps, bf16, 1 GPU",
                        "value": m["value"], "unit": "images/s", "dtype": "bf16",
                        "psnr_delta_db": (m.get("psnr") or {}).get("delta_db"),
                        "note": "the headline `value` is fp16 (the 16-bit mode that holds the 1e-3 dB bar); "
                                "bf16 misses it (DESIGN.md §5)"}
        lines = [x for x in args.lines.split(",") if x and x != "none"]
        if ws == 1 and args.model == "universal-ir" and lines:
            res["lines"] = []
            for x in lines:
                if x == "mixed8":
                    res["lines"].append(mixed_line(args, dev))
                    continue
                if x not in LINES:
                    raise SystemExit(f"bench: unknown line {x!r} (choose from {sorted(LINES) + ['mixed8']})")
                if LINES[x][3] == args.dtype and LINES[x][1] == args.res and LINES[x][2] == args.batch:
                    continue                       # that is the main line itself
                res["lines"].append(extra_line(args, x, dev))
        if ws == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args, synth.synth_state_dict(uspec, 0),
                                               synth.synth_state_dict(cspec, 0))
        print(json.dumps(res), flush=True)
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Throughput benchmark of the MI355X contrastive training step (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload: synthetic 10 s @ 16 kHz clips + 64-token clean and corrupted transcripts,
w2v-bert-2.0 Conformer + XLM-R-base text encoder with 3+3 unfrozen layers, bf16 MFMA / fp32
master weights.  One timed step = one optimizer step over the global batch:
    per micro-batch: GPU fbank from raw waveforms -> forward -> AlignmentAwareInfoNCE ->
    backward (gradients summed), then RCCL gradient all-reduce (N>1, overlapped with the last
    micro-batch's backward) -> clip_grad_norm_ + AdamW.
Training semantics with dropout on, layerdrop 0 and SpecAugment off, random-init
weights.

Batch (BASELINE configs): N=1 defaults to c2 (batch 64, one micro-batch); N>1 defaults to c3,
the global batch of 256 held fixed (strong scaling): local 256/N per rank in micro-batches of
at most 64 with gradient accumulation (2 x 64 at N=2, 64 at N=4, 32 at N=8), as SURVEY §8d asks
and the reference's batch/accumulation pair does (ref run_embedding_trainer_unfreeze.sh:9-34,
trainer_unfreeze.py:1064-1117).  --global-batch G overrides (e.g. 256 at N=1 = 4 x 64);
--batch B instead fixes the per-GPU batch (weak scaling).

--gpus N without torchrun: N ranks are spawned here (before anything touches the GPU), one per
GPU, rendezvous on 127.0.0.1.  Under torchrun WORLD_SIZE must equal N.

Rank 0 prints one JSON line.  `roofline` is for the dominant kernel (the bf16 GEMM
instantiation with the largest share of step time), timed per launch with HIP events on the
launch stream during the timed steps; `hbm_kernels` gives the achieved HBM GB/s of the fbank and
LayerNorm launches (same method); `cpu_baseline` times the oracle (CPU fp32 restatement of the
same step, oracle/) on the host at N=1, BASELINE.md §3 protocol.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BF16_PEAK_TFLOPS = 2516.6          # MI355X dense bf16 MFMA (256 CU x 4096 FLOP/clk x 2.4 GHz)
FP8_PEAK_TFLOPS = 5033.2           # dense MX-fp8 (scaled 16x16x128 f8f6f4: 2x the bf16 rate)
HBM_PEAK_GBPS = 8000.0             # MI355X HBM3E
GFLOP_PER_PAIR = {3: 1370.4, 5: 1429.5}   # SURVEY §8(d) algorithmic fwd+bwd FLOPs per pair (c2/c3, c4)
GFLOP_C5_PER_PAIR = 5999.6                 # c5 shape, 30 s clips, every encoder layer trainable
GFLOP_FWD_PER_PAIR = 641.8                 # SURVEY §8(d) forward only: 615.1 audio + 21.7 text + ≈5 heads


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)     # >= 20 timed steps after >= 5 warm-ups
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--global-batch", type=int, default=None,
                    help="global batch per optimizer step (default: 64 at N=1 = c2, 256 at N>1 = c3)")
    ap.add_argument("--micro-batch", type=int, default=64, help="largest per-GPU micro-batch")
    ap.add_argument("--batch", type=int, default=None, help="fixed local (per-GPU) batch: weak scaling")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--tokens", type=int, default=64)
    ap.add_argument("--unfreeze", type=int, default=3)
    ap.add_argument("--align", action="store_true", help="config 4: word-alignment head")
    ap.add_argument("--freeze", default="partial", choices=["partial", "none", "full"],
                    help="freeze_encoders (config 5 = none: every encoder layer trainable)")
    ap.add_argument("--fp8", action="store_true",
                    help="config 5's fp8 MFMA GEMMs: the Conformer forward GEMMs on MX-fp8 (e4m3, 32-k block scales)")
    ap.add_argument("--fp8-bwd", action="store_true",
                    help="with --fp8: the Conformer input-gradient GEMMs on MX-fp8 too (opt-in A/B; weight gradients stay bf16)")
    ap.add_argument("--overlap-optimizer", action="store_true",
                    help="clip + AdamW on a stream of their own, overlapped with the next step's forward "
                         "(TrainStep(overlap_optimizer=True); opt-in A/B, DESIGN §3)")
    ap.add_argument("--in-batch-weight", type=float, default=0.0,
                    help="optional in-batch-negative InfoNCE over the all-gathered global batch (0 = reference loss)")
    ap.add_argument("--eval", action="store_true",
                    help="time the forward-only evaluation step (SURVEY §8f rank 1, ref evaluate() :1165-1284): "
                         "GPU fbank -> forward without saved activations -> similarity + InfoNCE value")
    ap.add_argument("--audio-model", default="facebook/w2v-bert-2.0",
                    help="facebook/wav2vec2-base: the raw-waveform wav2vec2 encoder (SURVEY §8f rank 4, "
                         "not a BASELINE config: informational line, no CPU baseline)")
    ap.add_argument("--trace-steps", type=int, default=2,
                    help="extra (untimed) steps whose launches are timed with HIP events for roofline / hbm_kernels "
                         "(at least 1: the roofline object needs them)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=4, help="BASELINE.md §3: B=4")
    ap.add_argument("--cpu-steps", type=int, default=3, help="timed CPU steps (median), after 2 warm-ups")
    args = ap.parse_args(argv)
    if args.trace_steps < 1:
        ap.error("--trace-steps must be >= 1 (the roofline object is measured on those steps)")
    return args


def batch_plan(args, world):
    """-> (global batch, local batch, micro-batch, accumulation steps, scaling)."""
    if args.batch is not None:
        local = args.batch
        micro = min(local, args.micro_batch)
        scaling = "weak"
        glob = local * world
    else:
        glob = args.global_batch or (64 if world == 1 else 256)
        if glob % world:
            raise SystemExit(f"global batch {glob} does not split over {world} GPUs")
        local = glob // world
        micro = min(local, args.micro_batch)
        scaling = "strong"
    if local % micro:
        raise SystemExit(f"local batch {local} is not a multiple of the micro-batch {micro}")
    return glob, local, micro, local // micro, scaling


# ------------------------------------------------------------------ CPU baseline
def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cgroup_cpus():
    """CPUs the job may use under its cgroup CPU quota (cpu.max 'quota period'), or None."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                return max(1, int(int(q) // int(per)))
        except (OSError, ValueError):
            pass
    try:   # cgroup v1
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return max(1, q // per)
    except (OSError, ValueError):
        pass
    return None


def cpu_baseline(args):
    """the oracle (CPU fp32 restatement of the step, pinned to the reference by
    the golden fixtures) at c1 and c2 shapes with B=4, every host core this job may use, 2 warm-up
    steps then the median of >= 3 timed steps; the CPU model is reported."""
    import torch
    from oracle import fbank_ref, ref_model as R
    # every host core, torch.set_num_threads(len(os.sched_getaffinity(0))).  On the
    # GPU pool the affinity mask shows the whole machine (256 cores) while the job runs under a CPU
    # quota (cgroup cpu.max; OMP_NUM_THREADS is set to it): 256 torch threads on a 16-CPU quota did
    # not finish one warm-up step in 180 s (r3).  "Every host core" is therefore read as every core
    # the job may use: min(affinity, cgroup quota, OMP_NUM_THREADS — which the pool sets to the
    # quota); the affinity count is reported beside it.
    cores = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = min(cores, _cgroup_cpus() or cores, int(omp) if omp and omp.isdigit() else cores)
    torch.set_num_threads(threads)
    cfg = R.ModelCfg(use_word_alignment=args.align, text_layers_to_unfreeze=args.unfreeze,
                     audio_layers_to_unfreeze=args.unfreeze)
    shapes = R.param_shapes(cfg, spec_augment=False)
    trainable = R.trainable_names([n for n, _ in shapes], cfg)
    g = torch.Generator().manual_seed(0)
    p = {}
    for n, s in shapes:
        t = torch.randn(s, generator=g) * 0.02
        if n.endswith(".weight") and ("norm" in n.lower() or "LayerNorm" in n):
            t = torch.ones(s)
        p[n] = t.requires_grad_(n in trainable and not n.startswith("text_encoder.pooler"))
    m = {n: torch.zeros_like(t) for n, t in p.items() if t.requires_grad}
    v = {n: torch.zeros_like(t) for n, t in p.items() if t.requires_grad}

    def make_batch(B, N, L):
        feats = [fbank_ref.extract(fbank_ref.synth_wave(1000 + i, N))[0] for i in range(B)]
        f, am = fbank_ref.collate(feats)
        ids = torch.randint(5, 250000, (B, L))
        ids[:, 0], ids[:, -1] = 0, 2
        neg = ids.clone()
        neg[:, 1:max(2, L // 5)] = torch.randint(5, 250000, (B, max(2, L // 5) - 1))
        mask = torch.ones(B, L, dtype=torch.long)
        return {"input_ids_pos": ids, "attention_mask_pos": mask, "input_ids_neg": neg, "attention_mask_neg": mask,
                "input_values": torch.from_numpy(f), "attention_mask_audio": torch.from_numpy(am)}

    def one_step(step, B, N, L):
        if args.eval:
            with torch.no_grad():
                R.step_loss(p, make_batch(B, N, L), cfg)
            return
        batch = make_batch(B, N, L)   # numpy fbank inside the timed step, as the GPU step's fbank
        loss, *_ = R.step_loss(p, batch, cfg)
        loss.backward()
        with torch.no_grad():
            gs = [t.grad for t in p.values() if t.grad is not None]
            tot = torch.sqrt(sum((x.double() ** 2).sum() for x in gs)).item()
            coef = min(1.0, 1.0 / (tot + 1e-6))
            for n, t in p.items():
                if t.grad is None:
                    continue
                lr = 2.1e-3 / 50 if ("text_encoder" in n or "audio_encoder" in n) else 2.1e-3
                t2, m[n], v[n] = R.adamw_step(t, t.grad * coef, m[n], v[n], lr=lr, step=step)
                t.copy_(t2)
                t.grad = None

    def timed(B, seconds, L):
        N = int(seconds * 16000)
        for w in range(2):
            t0 = time.perf_counter()
            one_step(1 + w, B, N, L)
            print(f"[cpu_baseline] {seconds:g} s x {L} tok, B={B}: warm-up {w} {time.perf_counter() - t0:.2f} s",
                  file=sys.stderr, flush=True)
        dts = []
        for s in range(max(3, args.cpu_steps)):
            t0 = time.perf_counter()
            one_step(3 + s, B, N, L)
            dts.append(time.perf_counter() - t0)
            print(f"[cpu_baseline] {seconds:g} s x {L} tok, B={B}: step {s} {dts[-1]:.2f} s", file=sys.stderr,
                  flush=True)
        return statistics.median(dts)

    B = args.cpu_batch
    dt_c2 = timed(B, args.seconds, args.tokens)
    dt_c1 = timed(B, 2.0, 16) if not args.eval else None
    what = "forward-only evaluation step (numpy fbank + forward + loss, no_grad)" if args.eval else \
        "full train step incl. numpy fbank + clip + two-group AdamW"
    out = {"value": round(B / dt_c2, 4), "unit": "audio-text pairs/s", "cores": threads, "kind": "port",
           "cpu_model": _cpu_model(), "host_cores_visible": cores,
           "sample": f"oracle/ (CPU fp32 torch restatement, pinned to the reference by tests/golden) {what}; "
                     f"{args.seconds:g} s clips + {args.tokens}-token transcripts, {args.unfreeze} unfrozen layers, "
                     f"batch {B}; 2 warm-up steps, median of {max(3, args.cpu_steps)} timed steps = {dt_c2:.2f} s/step; "
                     f"threads = every host core this job may use: min(len(os.sched_getaffinity(0)) = {cores}, the "
                     f"cgroup CPU quota, OMP_NUM_THREADS) = {threads} (BASELINE.md §3)"}
    if dt_c1 is not None:
        out["c1"] = {"value": round(B / dt_c1, 4), "unit": "audio-text pairs/s",
                     "sample": f"c1 shapes: 2 s clips + 16-token transcripts, batch {B}, {dt_c1:.2f} s/step (median)"}
    return out


def hbm_traffic(kernel, c5=False):
    """Per-launch HBM bytes of `kernel` from the latest committed PMC reduction of the same
    workload family (profiles/rNN*_hbm_traffic.json, made by profiles/profile_bench.sh: separate
    rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this bench; gfx950 FETCH_SIZE x2 correction
    applied).  c5: the config-5 files (tag containing "c5"); otherwise the others."""
    import glob
    files = sorted(f for f in glob.glob(os.path.join(ROOT, "profiles", "r*_hbm_traffic.json"))
                   if ("c5" in os.path.basename(f)) == c5)
    if not files:
        return None, None
    # rocprofv3 names the 8-phase GEMM with its MX template argument (", false>"); the library's
    # kernel query omits it
    d = {k.replace(", false>", ">"): v for k, v in json.load(open(files[-1])).items()}
    if kernel not in d:
        return None, os.path.relpath(files[-1], ROOT)
    return d[kernel]["hbm_bytes_per_launch"], os.path.relpath(files[-1], ROOT)


# ---------------------------------------------------------------------- launcher
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawned(rank, world, port, argv):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), LOCAL_WORLD_SIZE=str(world))
    main(argv)


def launch(argv=None):
    args = parse(argv)
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
        return main(argv)
    if args.gpus == 1:
        return main(argv)
    # one process per GPU, started before this process touches the GPU
    import torch.multiprocessing as mp
    mp.start_processes(_spawned, args=(args.gpus, _free_port(), argv), nprocs=args.gpus, start_method="spawn")


# ------------------------------------------------------------------------- bench
def main(argv=None):
    args = parse(argv)
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("STE_BENCH_PLAN_ONLY") == "1":
        # launcher check without a GPU (tests/test_bench_cpu.py): rendezvous over gloo, report the plan
        if world > 1:
            dist.init_process_group("gloo")
            t = torch.ones(1)
            dist.all_reduce(t)
            assert int(t.item()) == world
        glob, lbatch, micro, acc, scaling = batch_plan(args, world)
        print(json.dumps({"rank": rank, "local_rank": local, "world": world, "global_batch": glob,
                          "local_batch": lbatch, "micro_batch": micro, "accumulation_steps": acc,
                          "scaling": scaling}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    # STE_BENCH_BACKEND=gloo with STE_BENCH_SHARE_GPU=1: rehearsal of the multi-rank flow with every
    # rank on GPU 0 (a one-GPU box); the measured runs use RCCL ("nccl"), one GPU per rank
    if os.environ.get("STE_BENCH_SHARE_GPU") == "1":
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        backend = os.environ.get("STE_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    from speech_transcript_embeddings_amd import ops
    from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
    from speech_transcript_embeddings_amd.train import TrainStep, synthetic_batch

    glob, lbatch, micro, acc, scaling = batch_plan(args, world)
    raw = "wav2vec2" in args.audio_model
    model = EnhancedAudioTextModel(use_word_alignment=args.align, text_layers_to_unfreeze=args.unfreeze,
                                   audio_layers_to_unfreeze=args.unfreeze, freeze_encoders=args.freeze,
                                   device=f"cuda:{local}", spec_augment=False,  # timed without SpecAugment
                                   fp8_gemm=args.fp8, audio_model_name=args.audio_model,
                                   audio_embedding_dim=768 if raw else 1024)
    model.audio_cfg.layerdrop = 0.0
    model.fp8_bwd = bool(args.fp8 and args.fp8_bwd)
    step = TrainStep(model, warmup=100, total_steps=100000, accumulation_steps=acc,
                     in_batch_weight=args.in_batch_weight, micro_batch=micro, max_text_length=args.tokens,
                     overlap_optimizer=args.overlap_optimizer)
    nsamp, L = int(args.seconds * 16000), args.tokens
    # resident synthetic inputs, a different shard per rank and micro-batch
    data = [synthetic_batch(micro, nsamp, L, device=f"cuda:{local}", seed=k, rank=rank) for k in range(acc)]
    if args.eval:
        from speech_transcript_embeddings_amd.evaluate import EvalStep
        model.eval()
        ev = EvalStep(model, 0.1, 0.5)

        def run():
            for wav, lens, ids_p, m_p, ids_n, m_n in data:
                feats, amask = step.features(wav, lens)
                sp, sn, lo = ev({"input_ids_pos": ids_p, "attention_mask_pos": m_p, "input_ids_neg": ids_n,
                                 "attention_mask_neg": m_n, "input_values": feats, "attention_mask_audio": amask})
                step.last = {"loss": lo, "s_pos": sp, "s_neg": sn}
    else:
        def run():
            for d in data:
                step(*d)
            assert step._micro == 0, "an optimizer step per timed step"

    # the step's own stream at the highest priority: the text encoder's side stream (normal
    # priority) then fills CUs the audio chain leaves idle instead of competing for them
    torch.cuda.synchronize()
    prio = os.environ.get("STE_MAIN_PRIORITY", "1") != "0"
    main_stream = torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1]) if prio else \
        torch.cuda.current_stream()
    with torch.cuda.stream(main_stream):
        for _ in range(args.warmup):
            run()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            run()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        # per-launch HIP-event timings (roofline, hbm_kernels) on extra steps of the same
        # workload after the timed ones: the ~1,200 event records per step slow the host's
        # enqueue, which keeps pace with the GPU only just (profiles/graph_probe.py), so they
        # stay out of the timed region
        ops.GEMM_TRACE, ops.HBM_TRACE = [], []
        for _ in range(args.trace_steps):
            run()
        torch.cuda.synchronize()
    trace, ops.GEMM_TRACE = ops.GEMM_TRACE, None
    htrace, ops.HBM_TRACE = ops.HBM_TRACE, None
    loss = float(step.last["loss"].item())
    if world > 1:
        t = torch.tensor([elapsed], device=f"cuda:{local}", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # dominant-kernel roofline from per-launch HIP event timings of the timed steps
    # launches on the step's own stream only: a side-stream launch (the text encoder) overlaps the
    # main stream, so its event interval includes time spent waiting for CUs
    own = main_stream.cuda_stream
    agg = {}
    for name, flops, e0, e1, _shape, sid in trace:
        if sid != own:
            continue
        a = agg.setdefault(name, [0, 0.0, 0.0])
        a[0] += 1
        a[1] += flops
        a[2] += e0.elapsed_time(e1) * 1e-3
    if not agg:
        raise SystemExit("bench: no GEMM launch was traced on the step's stream (--trace-steps must be >= 1)")
    dom = max(agg, key=lambda k: agg[k][2])
    n_l, fl, tm = agg[dom]
    achieved = fl / tm / 1e12
    gemm_time = sum(a[2] for a in agg.values()) / args.trace_steps
    hagg = {}
    # the optimizer's launches (Σg², AdamW) on its own stream with overlap_optimizer: they share
    # the chip with the next step's forward, so their event intervals are in-step times
    opt_sid = step._opt_stream.cuda_stream if getattr(step, "_opt_stream", None) is not None else None
    for name, nb, e0, e1, sid in htrace:
        if sid != own and not (sid == opt_sid and name in ("adamw", "sumsq")):
            continue
        a = hagg.setdefault(name, [0, 0.0, 0.0])
        a[0] += 1
        a[1] += nb
        a[2] += e0.elapsed_time(e1) * 1e-3
    hbm = {k: {"launches_per_step": n // args.trace_steps, "avg_launch_us": round(t_ / n * 1e6, 2),
               "algorithmic_mb_per_launch": round(b / n / 1e6, 3), "achieved_GBps": round(b / t_ / 1e9, 1),
               "frac_of_8TBps": round(b / t_ / 1e9 / HBM_PEAK_GBPS, 4), "ms_per_step": round(t_ / args.trace_steps * 1e3, 3)}
           for k, (n, b, t_) in sorted(hagg.items())}
    pairs = glob * args.steps / elapsed
    # SURVEY §8(d) algorithmic FLOPs per pair exist for the 10 s / 64-token configs c2/c3 (3
    # unfrozen layers) and c4 (5 + alignment head); other shapes report no step fraction
    known = args.seconds == 10.0 and args.tokens == 64 and args.freeze == "partial" and \
        (args.unfreeze, args.align) in ((3, False), (5, True))
    gflop = (GFLOP_FWD_PER_PAIR if args.eval else GFLOP_PER_PAIR[args.unfreeze]) if known else None
    c5 = args.seconds == 30.0 and args.tokens == 64 and args.freeze == "none" and not args.align and not args.eval
    if c5:
        gflop = GFLOP_C5_PER_PAIR
    if raw:
        cname = "wav2vec2-base raw-waveform encoder (SURVEY §8f rank 4, not a BASELINE config)"
        gflop = None
    elif args.seconds == 10.0 and args.freeze == "partial" and args.tokens == 64:
        cname = {(3, False): "c2" if (world == 1 and glob == 64) else "c3", (5, True): "c4"}.get(
            (args.unfreeze, args.align), "custom")
    elif args.freeze == "none":
        cname = ("c5-shape (bf16 GEMMs)" if not args.fp8 else
                 "c5-shape (MX-fp8 Conformer fwd + input-gradient GEMMs)" if args.fp8_bwd else
                 "c5-shape (MX-fp8 Conformer fwd GEMMs)")
    else:
        cname = "custom"
    peak = FP8_PEAK_TFLOPS if dom in ("gemm_mx8_kernel", "gemm_8ph_kernel<mx8>") else BF16_PEAK_TFLOPS
    traffic, traffic_src = hbm_traffic(dom, c5=c5)
    out = {
        "metric": ("evaluated audio–text pairs/sec, forward only (whole node), 10s@16kHz + 64-tok" if args.eval else
                   "audio–text pairs/sec (whole node), 10s@16kHz + 64-tok, 1/2/4/8 MI355X"),
        "value": round(pairs, 3), "unit": "pairs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": scaling,
        "vs_baseline": None, "dtype": ("bf16" if not args.fp8 else
                                       "bf16 + mxfp8-e4m3 (Conformer fwd + dX GEMMs)" if args.fp8_bwd else
                                       "bf16 + mxfp8-e4m3 (Conformer fwd GEMMs)"),
        "data": "synthetic (SURVEY §8d waveforms + token ids), random-init weights",
        "config": {"workload": f"{cname}: global batch {glob} = {world} GPU x {acc} micro-batch(es) of {micro} pairs, "
                               f"each pair {args.seconds:g}s@16kHz audio + {L}-tok clean + {L}-tok corrupt; "
                               + ("wav2vec2-base (conv stack + pos conv + 12L) + XLM-R-base 12L, " if raw else
                                  "w2v-bert-2.0 Conformer 24L + XLM-R-base 12L, ")
                               + f"{'all layers trainable' if args.freeze == 'none' else f'{args.unfreeze}+{args.unfreeze} unfrozen'}"
                               f"{', alignment head' if args.align else ''}; {'GPU wave normalisation' if raw else 'GPU fbank'} -> "
                               + ("fwd (no saved activations, eval mode) -> similarity + InfoNCE value" if args.eval
                                  else "fwd -> InfoNCE -> bwd -> allreduce -> clip+AdamW"),
                   "global_batch": glob, "local_batch": lbatch, "micro_batch": micro, "accumulation_steps": acc,
                   "seq_len_audio_frames": (model.audio_cfg.frames(nsamp)[-1] if raw else
                                            ((1 + (nsamp - 400) // 160) + 1) // 2),
                   "seq_len_text": L, "parallelism": f"dp{world}"},
        "step_roofline_frac": round(pairs * gflop / (world * BF16_PEAK_TFLOPS * 1e3), 4) if gflop else None,
        # c5 with --fp8: also against the dense MX-fp8 peak (839 pairs/s per GPU)
        **({"step_roofline_frac_fp8_peak": round(pairs * gflop / (world * FP8_PEAK_TFLOPS * 1e3), 4)}
           if (gflop and c5 and args.fp8) else {}),
        "gflop_per_pair": gflop,
        "roofline": {"bound": "mfma", "kernel": dom, "launches_per_step": n_l // args.trace_steps,
                     "achieved": round(achieved, 1), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(achieved / peak, 4), "traffic": traffic,
                     "traffic_unit": "HBM bytes per launch", "traffic_source": traffic_src,
                     "avg_launch_us": round(tm / n_l * 1e6, 2), "algorithmic_gflop_per_launch": round(fl / n_l / 1e9, 3),
                     "gemm_ms_per_step_all_variants": round(gemm_time * 1e3, 2),
                     "timing": f"HIP events per launch on the launch stream, {args.trace_steps} traced steps after the timed ones; main-stream launches only"},
        "hbm_kernels": hbm,
        "loss": round(loss, 5),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not raw:
        out["cpu_baseline"] = cpu_baseline(args)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    launch()

"""Benchmark: swapped 256x256 frames/s of GHOST's swap forward on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W --batch 64 --backbone unet --num-blocks 2]
    torchrun --nproc-per-node N bench.py --gpus N ...     (driver's multi-GPU form)

One step = one faceshifter_batch of B synthetic aligned-face crops per GPU, device-resident:
uint8 BGR crops -> normalise -> AEI_Net (encoder + AAD generator, bf16) -> tanh -> uint8 BGR,
then (N > 1) an RCCL all-gather of every rank's swapped crops (frame order = rank order).
Weak scaling: B frames per GPU; value = N*B*K / max-over-ranks wall time of the K timed steps.

Besides the JSON line's throughput, it reports
* roofline: the dominant AAD kernel, aad_v4_kernel<64,2,true> (the two AADLayers of AADBlk8 that
  read the same h_in / z_attr at 256x256, h_in sampled through the bilinear x2 upsample of AADBlk7's
  128x128 output), HBM-bound: its algorithmic bytes per launch by SURVEY.md §8d's formula (fixed
  regardless of fusion: sum over its two AADLayers of |h_in| + |z_attr| + |out|, 64 frames at
  256x256x64 bf16 = 3.22 GB) / its average launch time, timed with HIP events recorded around each of its
  launches on the launch stream inside the timed region; `traffic` = PMC-measured HBM bytes per
  launch of the same kernel from profiles/traffic_latest.json;
* roofline_conv3x3 (MFMA-bound, all generator 3x3 convs) and aad_decoder_gbs (SURVEY.md §8d
  definition: 135.58 MB/frame of AADLayer bytes / total AAD kernel time);
* cpu_baseline: the CPU restatement (oracle/aei_ref.py, fp32, same ATen op sequence as the
  reference) on this host's cores over a bounded sample (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

try:
    BASELINE_METRIC = json.load(open(os.path.join(REPO, "BASELINE.json")))["metric"]
except (OSError, ValueError, KeyError):
    BASELINE_METRIC = "swapped frames/sec at 256\u00d7256 bf16, 1/2/4/8 MI355X; AAD decoder HBM GB/s"
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
BF16_PEAK_TFLOPS = 2500.0    # dense bf16 MFMA spec
AAD_BYTES_PER_FRAME = {"unet": 135.58e6, "linknet": 156.02e6, "resnet": 135.58e6}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="frames per GPU per step")
    ap.add_argument("--backbone", default="unet")
    ap.add_argument("--num-blocks", type=int, default=2)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget (0 = skip)")
    ap.add_argument("--no-profile", action="store_true", help="skip the per-kernel HIP-event timing")
    ap.add_argument("--arc-batch", type=int, default=64,
                    help="faces per ArcFace (iresnet100) embedding batch in the side measurement (0 = skip)")
    return ap.parse_args()


def pmc_traffic(kernel_substr):
    """HBM bytes per launch of a kernel from the committed PMC summary (tools/pmc_traffic.py over
    separate rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this bench, gfx950 FETCH x2 correction)."""
    path = os.path.join(REPO, "profiles", "traffic_latest.json")
    try:
        data = json.load(open(path))
    except (OSError, ValueError):
        return None
    for k in data.get("kernels", []):
        if kernel_substr in k["kernel"] and k.get("hbm_bytes"):
            return {"bytes_per_launch": k["hbm_bytes"], "read": k["read_bytes"], "write": k["write_bytes"],
                    "source": "profiles/traffic_latest.json (" + data.get("source", "rocprofv3 --pmc") + ")"}
    return None


def arcface_flops_per_face(layers=(3, 13, 30, 3)):
    """2*MAC of IResNet at 112x112: stem, per block conv1 (s1) + conv2 (stride) + downsample, fc."""
    fl = 2.0 * 112 * 112 * 64 * 27
    inp, H = 64, 112
    for planes, n in zip((64, 128, 256, 512), layers):
        for b in range(n):
            s = 2 if b == 0 else 1
            Ho = H // s
            fl += 2.0 * H * H * planes * 9 * inp + 2.0 * Ho * Ho * planes * 9 * planes
            if b == 0:
                fl += 2.0 * Ho * Ho * planes * inp
            inp, H = planes, Ho
    return fl + 2.0 * 512 * 49 * 512


def arcface_leg(dev, n, steps):
    """Side measurement (not the headline): iresnet100 bf16 embeddings/s on device u8 224x224 crops
    (normalise + 0.5x resize + network), the per-frame identity path of config 5."""
    from ghost_amd.arcface import iresnet100
    from oracle.arcface_ref import make_weights, param_specs
    net = iresnet100(fp16=False, compute_dtype=torch.bfloat16).eval()
    net.load_state_dict(make_weights(param_specs()))
    net = net.to(dev)
    crops = torch.from_numpy(np.random.Generator(np.random.PCG64(5)).integers(0, 256, (n, 224, 224, 3),
                                                                           dtype=np.uint8)).to(dev)
    for _ in range(2):
        net.embed_u8(crops)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        net.embed_u8(crops)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    fl = arcface_flops_per_face() * n
    return {"model": "iresnet100 bf16 (synthetic weights), u8 224x224 crops -> 512-d embeddings", "batch": n,
            "ms_per_batch": round(ms, 3), "embeddings_per_s": round(n / (ms / 1e3), 1),
            "gflop_per_face": round(arcface_flops_per_face() / 1e9, 2),
            "mfma_tflops": round(fl / (ms / 1e3) / 1e12, 1),
            "mfma_frac": round(fl / (ms / 1e3) / 1e12 / BF16_PEAK_TFLOPS, 4)}


def cpu_baseline(backbone, nb, seconds):
    """Oracle (CPU fp32 restatement) frames/s on this host, bounded sample."""
    from oracle import aei_ref
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    p = aei_ref.make_weights(aei_ref.param_specs(backbone, nb))
    bs = 4
    xt, z = aei_ref.make_inputs(bs, seed=3)
    aei_ref.aei_forward(p, xt[:1], z[:1], backbone, nb)       # warm-up
    frames, t0 = 0, time.perf_counter()
    while True:
        aei_ref.aei_forward(p, xt, z, backbone, nb)
        frames += bs
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": round(frames / el, 3), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{frames} frames of {backbone}/{nb} fp32 in batches of {bs} (oracle/aei_ref.py), {el:.1f}s"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from ghost_amd.network import AEI_Net
    from oracle.aei_ref import make_weights, param_specs   # deterministic synthetic weights (no checkpoint offline)

    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    G = AEI_Net(a.backbone, num_blocks=a.num_blocks, c_id=512, compute_dtype=dt).eval()
    G.load_state_dict(make_weights(param_specs(a.backbone, a.num_blocks)))
    G = G.to(dev)

    B = a.batch
    rng = np.random.Generator(np.random.PCG64(1000 + rank))
    crops = torch.from_numpy(rng.integers(0, 256, size=(B, 256, 256, 3), dtype=np.uint8)).to(dev)
    z = torch.from_numpy(np.random.Generator(np.random.PCG64(1)).normal(size=(1, 512)).astype(np.float32)).to(dev)
    # swap -> all-gather of the uint8 swaps to every rank; the gather of step k overlaps step k + 1
    # (dp.GatherPipeline; GHOST_DP_OVERLAP=0 gathers synchronously after each step)
    from ghost_amd.inference.dp import GatherPipeline
    pipe = GatherPipeline(lambda c, o: G.swap_u8(c, z, out=o), (B, 256, 256, 3), dev,
                          depth=2 if os.environ.get("GHOST_DP_OVERLAP", "1") != "0" else 1)

    def step():
        slot = pipe.submit(crops)
        if pipe.depth == 1:
            pipe.result(slot)

    for _ in range(a.warmup):
        step()
    pipe.drain()
    torch.cuda.synchronize()
    prof = not a.no_profile
    names = ["aad_all", "aad_dual_256", "conv3x3_all", "conv3x3_256", "in_stats_mask", "encoder", "upsample",
             "id_proj"]
    classes = {}
    if prof:
        # inside the timed region only the roofline kernel is bracketed (one HIP event pair per step,
        # recorded on the launch stream around each of its launches)
        G.profile(1 << names.index("aad_dual_256"))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    pipe.drain()                  # every step's all-gather is inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if prof:
        classes["aad_dual_256"] = G.profile_read(names.index("aad_dual_256"))
        # per-class breakdown from a separate, untimed pass (every kernel class bracketed)
        G.profile(0xFF)
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        for i, n in enumerate(names):
            if n != "aad_dual_256":
                classes[n] = G.profile_read(i)
        G.profile(0)

    if rank == 0:
        frames = world * B * a.steps
        value = frames / el
        res = {
            "metric": BASELINE_METRIC,
            "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(el / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": a.dtype if a.dtype == "fp32" else "bf16", "data": "synthetic",
            "config": {"workload": f"batch={B} synthetic 256x256 aligned faces per GPU, AEI_Net {a.backbone} "
                                   f"num_blocks={a.num_blocks}, faceshifter_batch (u8 in -> u8 out)"
                                   + (", RCCL all-gather of swapped crops" if world > 1 else ""),
                       "global_batch": world * B, "per_gpu_batch": B, "backbone": a.backbone,
                       "num_blocks": a.num_blocks, "parallelism": f"dp{world}"},
        }
        if prof and classes["aad_dual_256"]["launches"]:
            c = classes["aad_dual_256"]
            per_launch_bytes = c["bytes"] / c["launches"]
            per_launch_s = c["ms"] / c["launches"] / 1e3
            ach = per_launch_bytes / per_launch_s / 1e9
            ca8 = 32 if a.backbone == "linknet" else 64     # z_attr8 channels (AEI_Net.py:110,118)
            # layers in the kernel: the formula bytes per launch are L * B*256^2*(2*64 + Ca)*2
            nl = max(1, round(per_launch_bytes / (B * 65536 * (2 * 64 + ca8) * 2)))
            kname = f"aad_v4_kernel<{ca8}, {nl}, true>"
            what = ("two AADLayers sharing h_in/z_attr" if nl == 2 else
                    "the first AADLayer (its last_add_block partner runs in the fused tail)")
            res["roofline"] = {"kernel": f"{kname}: AADBlk8's block-input AAD kernel at 256x256, {what}, h_in = "
                                         "bilinear x2 of the 128x128 block output sampled in-kernel (IN-normalise, "
                                         "sigmoid mask, MFMA gamma/beta, blend, ReLU), next tile in flight",
                               "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": pmc_traffic(kname),
                               "bytes_note": "achieved counts SURVEY.md 8d bytes (|h_in|+|z_attr|+|out| per AADLayer, "
                                             "h_in at 256x256); the kernel physically moves the 128x128 h_in once "
                                             "for both layers: see physical_gbs / traffic",
                               "bytes_per_launch": per_launch_bytes, "avg_launch_us": round(per_launch_s * 1e6, 2),
                               "launches_timed": c["launches"]}
            tr = res["roofline"]["traffic"]
            if tr:
                res["roofline"]["physical_gbs"] = round(tr["bytes_per_launch"] / per_launch_s / 1e9, 1)
                res["roofline"]["physical_frac"] = round(res["roofline"]["physical_gbs"] / HBM_PEAK_GBS, 4)
            cc = classes["conv3x3_all"]
            if cc["launches"]:
                tf = cc["flops"] / (cc["ms"] / 1e3) / 1e12
                res["roofline_conv3x3"] = {"bound": "mfma", "achieved": round(tf, 1), "peak": BF16_PEAK_TFLOPS,
                                           "unit": "TFLOP/s", "frac": round(tf / BF16_PEAK_TFLOPS, 4)}
            aad = classes["aad_all"]
            if aad["ms"]:
                # SURVEY.md §8d definition: sum over AADLayers of |h_in|+|z_attr|+|out| / AAD kernel time
                res["aad_decoder_gbs"] = round(AAD_BYTES_PER_FRAME[a.backbone] * B * a.steps
                                               / (aad["ms"] / 1e3) / 1e9, 1)
                res["aad_decoder_hbm_frac"] = round(res["aad_decoder_gbs"] / HBM_PEAK_GBS, 4)
            res["kernel_ms_per_step"] = {k: round(v["ms"] / a.steps, 3) for k, v in classes.items()}
            res["kernel_ms_per_step_note"] = ("aad_dual_256 from the timed region; the other classes from an "
                                              "untimed pass with every class bracketed by HIP events")
        if world == 1 and a.arc_batch > 0:
            res["arcface"] = arcface_leg(dev, a.arc_batch, max(3, a.steps // 2))
        if world == 1 and a.cpu_seconds > 0:
            res["cpu_baseline"] = cpu_baseline(a.backbone, a.num_blocks, a.cpu_seconds)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

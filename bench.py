"""Benchmark: swapped 256x256 frames/s of GHOST's swap forward on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W --batch 64 --backbone unet --num-blocks 2 --identities 1]
    torchrun --nproc-per-node N bench.py --gpus N ...     (driver's multi-GPU form)

Headline (BASELINE config 2 at N = 1, config 4 at N > 1): one step = one faceshifter_batch of B
synthetic aligned-face crops per GPU, device-resident: uint8 BGR crops -> normalise -> AEI_Net
(encoder + AAD generator, bf16) -> tanh -> uint8 BGR, then (N > 1) an RCCL all-gather of every
rank's swapped crops (frame order = rank order).  Weak scaling: B frames per GPU;
value = N*B*K / max-over-ranks wall time of the K timed steps.  ``--identities 4 --backbone linknet
--num-blocks 3`` makes the headline BASELINE config 5 (mixed-identity batches, per-sample identity
rows).

Besides the JSON line's throughput, rank 0 at N = 1 reports
* roofline: the dominant AAD kernel, aad_v5_kernel<__bf16,64,2,true,2,true> (the two AADLayers of AADBlk8
  that read the same h_in / z_attr at 256x256, h_in sampled through the bilinear x2 upsample of AADBlk7's
  128x128 output; one of them writes the 3x3 RGB conv's tap partials), HBM-bound.  ``achieved`` = the bytes
  that fused kernel must move at minimum (the 128x128 source of h_in once, z_attr8 once, its outputs as
  stored: 1.476 GB at B = 64) / its average launch duration in the timed configuration — the committed
  rocprofv3 trace row of that symbol (profiles/rNN_kernel_stats.csv, tools/profile_round.sh runs this same
  command under rocprofv3), with the live in-kernel clock of the timed region beside it (live_clock_us);
  ``traffic`` = its PMC-measured HBM bytes per launch (profiles/rNN_traffic.json); ``fractions`` gives the
  minimum-bytes, physical (PMC) and SURVEY.md §8d per-layer-formula (|h_in|+|z_attr|+|out| per AADLayer,
  3.22 GB: bytes the fused kernel never moves) fractions side by side; ``isolated`` the same kernel one
  batch at a time (live clock and the one-stream trace row);
* roofline_conv3x3 (MFMA-bound, all generator 3x3 convs) and aad_decoder_gbs (SURVEY.md §8d
  definition: AADLayer bytes / total AAD kernel time);
* legs: the D2H-inclusive config 2 (pinned host output, copy overlapped with the next batch), config 5
  (4 identities, linknet/3, mixed batches), config 3 (a 900-frame 1080p video: H2D of the crops,
  BS-batched swaps with per-batch D2H, `present` re-insertion, H2D of the full frames, paste-back
  blend, D2H of the blended frames), ArcFace embeddings/s;
* cpu_baseline: the CPU restatement (oracle/aei_ref.py, fp32, same ATen op sequence as the
  reference) on this host's CPUs at B = 1 and B = 64, 1 warm-up + 3 timed iterations each.
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

from ghost_amd.inference.streams import stream_set  # noqa: E402

try:
    BASELINE_METRIC = json.load(open(os.path.join(REPO, "BASELINE.json")))["metric"]
except (OSError, ValueError, KeyError):
    BASELINE_METRIC = "swapped frames/sec at 256×256 bf16, 1/2/4/8 MI355X; AAD decoder HBM GB/s"
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
BF16_PEAK_TFLOPS = 2500.0    # dense bf16 MFMA spec
AAD_BYTES_PER_FRAME = {"unet": 135.58e6, "linknet": 156.02e6, "resnet": 135.58e6}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="frames per GPU per step")
    ap.add_argument("--backbone", default="unet")
    ap.add_argument("--num-blocks", type=int, default=2)
    ap.add_argument("--identities", type=int, default=1, help="source identities mixed in every batch (config 5: 4)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--legs", default="config5_multi,per_batch_projection,d2h,fp16,config5,video,latency,arcface",
                    help="side measurements (comma list of config5_multi (every N), per_batch_projection, d2h, fp16, "
                         "config5, video, latency, arcface (N = 1 only); '' = none)")
    ap.add_argument("--c5-frames", type=int, default=240, help="video frames per GPU of the config5_multi leg")
    ap.add_argument("--video", type=int, default=900, help="frames of the config-3 video leg")
    ap.add_argument("--cpu-batches", default="1,64", help="CPU baseline batch sizes ('' = skip)")
    ap.add_argument("--no-profile", action="store_true", help="skip the per-kernel HIP-event timing")
    ap.add_argument("--arc-batch", default="256,128",
                    help="faces per ArcFace embedding launch in its leg (comma list; the first is the leg's headline)")
    ap.add_argument("--streams", type=int, default=2,
                    help="batches in flight on the GPU (dp.GatherPipeline streams; 1 = one batch at a time)")
    ap.add_argument("--opt", action="append", default=[],
                    help="AEI_Net plan option name=value (A/B runs), e.g. --opt fuse_stats=0")
    # the launcher's CPU rehearsal (tests/test_dp_cpu.py): gloo ranks on the CPU with a stand-in swap, the same
    # timed region / record / relay as the GPU run
    ap.add_argument("--standin-cpu", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


_MANGLED_TYPES = {"__bf16": "DF16b", "_Float16": "DF16_", "float": "f"}


def mangle(kname):
    """'aad_v5_kernel<__bf16, 64, 2, true, 2, true>' -> 'aad_v5_kernelIDF16bLi64ELi2ELb1ELi2ELb1EE' (the Itanium
    template-argument part of the symbol rocprofv3 records)."""
    import re
    m = re.match(r"(\w+)<(.*)>", kname)
    if not m:
        return None
    base, targs = m.group(1), [t.strip() for t in m.group(2).split(",")]
    enc = []
    for t in targs:
        if t in _MANGLED_TYPES:
            enc.append(_MANGLED_TYPES[t])
        elif t in ("true", "false"):
            enc.append("Lb1E" if t == "true" else "Lb0E")
        else:
            enc.append(f"Li{t}E")
    return base + "I" + "".join(enc) + "E"


def pmc_traffic(kname):
    """HBM bytes per launch of a kernel from the committed PMC summary (tools/pmc_traffic.py over
    separate rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this bench, gfx950 FETCH x2 correction)."""
    import glob
    rounds = sorted(glob.glob(os.path.join(REPO, "profiles", "r[0-9][0-9]_traffic.json")))
    if not rounds:
        return None
    path = rounds[-1]
    try:
        data = json.load(open(path))
    except (OSError, ValueError):
        return None
    rel = os.path.relpath(path, REPO)
    key = mangle(kname) or kname
    for k in data.get("kernels", []):
        if key in k["kernel"] and k.get("hbm_bytes"):
            return {"bytes_per_launch": k["hbm_bytes"], "read": k["read_bytes"], "write": k["write_bytes"],
                    "source": rel + " (" + data.get("source", "rocprofv3 --pmc") + ")"}
    return None


def mfma_profile(match=None):
    """The newest committed MFMA-utilisation summary (profiles/rNN_mfma.json, tools/pmc_mfma.sh: rocprofv3 --pmc
    SQ_VALU_MFMA_BUSY_CYCLES / SQ_INSTS_MFMA / SQ_INSTS_VALU / GRBM_GUI_ACTIVE ... over this bench's one-stream
    configuration and the ArcFace leg).  match: a kernel-name substring -> that kernel's rows only."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r[0-9][0-9]_mfma.json")))
    if not files:
        return None
    try:
        d = json.load(open(files[-1]))
    except (OSError, ValueError):
        return None
    out = {"source": os.path.relpath(files[-1], REPO), "definition": d.get("definitions", {}).get("mfma_busy")}
    for part in ("generator", "arcface"):
        if part not in d:
            continue
        rows = d[part]["kernels"]
        if match:
            rows = [r for r in rows if match in r["kernel"]]
        out[part] = {"totals": d[part]["totals"],
                     "kernels": [{k: r.get(k) for k in ("kernel", "grid", "dispatches", "mfma_busy", "valu_per_mfma",
                                                        "wait_frac", "eff_clock_ghz")} for r in rows[:12]]}
    return out


def rocprof_avg_us(kname):
    """The kernel's average duration in the newest committed rocprofv3 --stats summaries: the timed
    configuration (profiles/rNN_kernel_stats.csv: bench.py's two batches in flight) and one batch at a time
    (profiles/rNN_kernel_stats_1stream.csv).  kname: the demangled 'aad_v5_kernel<64, 2, true, 2>'."""
    import csv
    import glob
    mangled = mangle(kname)
    if not mangled:
        return None
    out = {}
    for key, pat in (("timed", "r[0-9][0-9]_kernel_stats.csv"), ("isolated", "r[0-9][0-9]_kernel_stats_1stream.csv")):
        files = sorted(glob.glob(os.path.join(REPO, "profiles", pat)))
        if not files:
            continue
        try:
            for r in csv.DictReader(open(files[-1])):
                nm = r.get("Name") or r.get("KernelName") or ""
                if mangled in nm or kname in nm.replace("ghost::", ""):
                    out[key + "_avg_us"] = round(float(r["AverageNs"]) / 1e3, 2)
                    out[key + "_calls"] = int(r["Calls"])
                    out[key + "_source"] = os.path.relpath(files[-1], REPO)
                    break
        except (OSError, ValueError, KeyError):
            continue
    return out or None


def aad_v4_min_bytes(B, ca8, nl, num_blocks, tap_partials):
    """Minimum HBM bytes of one aad_v4 launch (AADBlk8's block-input AADLayer pair at 256x256, bf16): the
    128x128x64 h_in source once, z_attr8 (ca8 channels) once, and each of the nl outputs as stored — 64 bf16
    channels, or the 15 fp16 per pixel of row-summed tap partials (ghost_amd/csrc/tap_rows.h) for a layer that
    feeds the 3x3 conv to RGB through them
    (GHOST_AEI_OPT_TAP_PARTIALS: nb >= 2 -> last_add_block's layer in mode 2; nb = 1 -> the h path's layer in
    modes 1 and 2, last_add_block's in mode 2).  Returns (bytes, layers writing partials, the kernel's ZPM mask)."""
    if num_blocks >= 2:
        zpm = 2 if tap_partials == 2 else 0
    else:
        zpm = {0: 0, 1: 1, 2: 3}.get(tap_partials, 0)
    n_part = min(nl, bin(zpm).count("1"))
    return B * (128 * 128 * 64 + 65536 * ca8 + (nl - n_part) * 65536 * 64 + n_part * 65536 * 15) * 2.0, n_part, zpm


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


def make_model(backbone, nb, dt, dev):
    from ghost_amd.network import AEI_Net
    from oracle.aei_ref import make_weights, param_specs   # deterministic synthetic weights (no checkpoint offline)
    G = AEI_Net(backbone, num_blocks=nb, c_id=512, compute_dtype=dt).eval()
    G.load_state_dict(make_weights(param_specs(backbone, nb)))
    return G.to(dev)


def identity_rows(n, dev):
    return torch.from_numpy(np.random.Generator(np.random.PCG64(1)).normal(size=(n, 512)).astype(np.float32)).to(dev)


def compute_streams(dev, n):
    """The compute streams of n batches in flight: the caller's stream, then the device StreamSet's (streams.py: one
    fixed set of streams per process, so no leg adds hardware-queue sharing for the legs after it)."""
    ss = stream_set(dev)
    return [torch.cuda.current_stream(dev)] + [ss.compute(i) for i in range(1, max(1, n))]


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


# ---------------------------------------------------------------------------------------------
# side legs (rank 0, N = 1)
# ---------------------------------------------------------------------------------------------
def arcface_leg(dev, n, steps, nstreams=1):
    """iresnet100 bf16 embeddings/s on device u8 224x224 crops (normalise + 0.5x resize + network),
    the per-frame identity path of config 5.  Parity of the network itself is unpinned (the IResNet
    source and weights are not in the reference tree).  nstreams > 1: consecutive batches on that many
    streams (batches in flight, as the headline loop)."""
    from ghost_amd.arcface import iresnet100
    from oracle.arcface_ref import make_weights, param_specs
    net = iresnet100(fp16=False, compute_dtype=torch.bfloat16).eval()
    net.load_state_dict(make_weights(param_specs()))
    net = net.to(dev)
    crops = torch.from_numpy(np.random.Generator(np.random.PCG64(5)).integers(0, 256, (n, 224, 224, 3),
                                                                           dtype=np.uint8)).to(dev)
    main = torch.cuda.current_stream(dev)
    comp = compute_streams(dev, nstreams)
    for c in comp[1:]:
        c.wait_stream(main)
    k = [0]

    def step():
        with torch.cuda.stream(comp[k[0] % len(comp)]):
            net.embed_u8(crops)
        k[0] += 1

    el = timed(step, steps, 2)
    ms = el * 1e3 / steps
    fl = arcface_flops_per_face() * n
    return {"model": "iresnet100 bf16 (synthetic weights), u8 224x224 crops -> 512-d embeddings", "batch": n,
            "batches_in_flight": len(comp),
            "parity": "unpinned (no IResNet source, weights or fixtures in the reference)",
            "ms_per_batch": round(ms, 3), "embeddings_per_s": round(n / (ms / 1e3), 1),
            "gflop_per_face": round(arcface_flops_per_face() / 1e9, 2),
            "mfma_tflops": round(fl / (ms / 1e3) / 1e12, 1),
            "mfma_frac": round(fl / (ms / 1e3) / 1e12 / BF16_PEAK_TFLOPS, 4)}


def fp16_leg(dev, crops, z, steps, warmup, backbone, nb, nstreams=1):
    """Config 2 with the reference's own GPU precision: the module .half()'d after loading its weights
    (inference.py:27-30), fp16 crops' identity row (core.py:20-21): fp16 storage kernels
    (v_mfma_f32_16x16x32_f16), about 4x closer to the fp32 forward than bf16 storage."""
    from ghost_amd.network import AEI_Net
    from oracle.aei_ref import make_weights, param_specs
    G = AEI_Net(backbone, num_blocks=nb, c_id=512).eval()
    G.load_state_dict(make_weights(param_specs(backbone, nb)))
    G = G.to(dev).half()
    zh = z.half()
    table = G.identity_table(zh)               # the identity's projections once (as the headline)
    idx = torch.zeros(crops.shape[0], dtype=torch.int32, device=dev)
    B = crops.shape[0]
    ns = max(1, nstreams)
    outs = [torch.empty(B, 256, 256, 3, dtype=torch.uint8, device=dev) for _ in range(ns)]
    main = torch.cuda.current_stream(dev)
    comp = compute_streams(dev, ns)
    for c in comp[1:]:
        c.wait_stream(main)
    k = [0]

    def step():
        i = k[0] % ns
        with torch.cuda.stream(comp[i]):
            G.swap_u8_indexed(crops, table, idx, out=outs[i])
        k[0] += 1

    el = timed(step, steps, warmup)
    del G
    torch.cuda.empty_cache()
    return {"workload": f"config 2 with a .half() module: batch={B} {backbone}/{nb} fp16 storage (fp32 accumulation), "
                        f"u8 in -> u8 out, {ns} batch(es) in flight",
            "dtype": "f16", "frames_per_s": round(B * steps / el, 1), "ms_per_batch": round(el * 1e3 / steps, 3)}


def per_batch_projection_leg(G, crops, zs, idx, steps, warmup, nstreams):
    """The headline step without the identity table: the literal faceshifter_batch work of
    utils/inference/faceshifter_run.py:15-19 — the source embedding repeated over the batch (B rows, :15-16) and
    every AADLayer's fc1/fc2 plus up1 projected from those rows in every batch (AEI_Net.swap_u8), same crops,
    same batches in flight.  The bytes equal the headline's (tests/test_gpu_pipeline.py)."""
    from ghost_amd.inference.dp import GatherPipeline
    dev = crops.device
    B = crops.shape[0]
    zrows = zs.index_select(0, idx.long()).contiguous()

    def swap(c, o):
        return G.swap_u8(c, zrows, out=o)
    pipe = GatherPipeline(swap, (B, 256, 256, 3), dev, depth=2, streams=max(1, nstreams))
    el = timed_region(lambda: pipe.submit(crops), pipe.drain, steps, warmup, 1, dev)
    return {"workload": f"config 2 with per-batch identity projections: batch={B}, z_id rows repeated over the batch "
                        f"and fc1/fc2/up1 computed in every step (faceshifter_run.py:15-19), u8 in -> u8 out, "
                        f"{pipe.nstreams} batch(es) in flight",
            "frames_per_s": round(B * steps / el, 1), "ms_per_batch": round(el * 1e3 / steps, 3)}


def d2h_leg(swap, crops, steps, nstreams=1):
    """Config 2 including faceshifter_run.py:22's .cpu(): each batch's uint8 swaps are copied into a
    pinned host buffer on a copy stream while the next batch is swapped (two device/host slots); with
    nstreams = 2 consecutive batches are swapped on two compute streams (two batches in flight, as the
    headline loop)."""
    dev = crops.device
    B = crops.shape[0]
    outs = [torch.empty(B, 256, 256, 3, dtype=torch.uint8, device=dev) for _ in range(2)]
    hosts = [torch.empty(B, 256, 256, 3, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    copy = stream_set(dev).d2h
    main = torch.cuda.current_stream(dev)
    comp = compute_streams(dev, nstreams)
    for c in comp[1:]:
        c.wait_stream(main)
    done = [torch.cuda.Event() for _ in range(2)]
    copied = [None, None]
    k = [0]

    def step():
        s = k[0] % 2
        cur = comp[k[0] % len(comp)]
        if copied[s] is not None:
            cur.wait_event(copied[s])          # the copy still reading this slot
        with torch.cuda.stream(cur):
            swap(crops, outs[s])
        done[s].record(cur)
        with torch.cuda.stream(copy):
            copy.wait_event(done[s])
            hosts[s].copy_(outs[s], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(copy)
            copied[s] = ev
        k[0] += 1

    def run():
        step()

    # three timed windows of max(steps, 60) batches after the warm-up, median reported (one 20-batch window is
    # 0.12 s: short enough for host-side hiccups to move it by 10 %)
    n = max(steps, 60)
    els = []
    for w in range(3):
        els.append(timed(run, n, 3 if w == 0 else 0))
        copy.synchronize()
    el = float(np.median(els))
    return {"workload": f"config 2 + D2H: batch={B} unet/2 bf16 swaps copied to pinned host memory per batch "
                        f"(copy stream, overlapped with the next batch's swap; {len(comp)} batch(es) in flight)",
            "frames_per_s": round(B * n / el, 1), "ms_per_batch": round(el * 1e3 / n, 3),
            "windows_frames_per_s": [round(B * n / e, 1) for e in els], "batches_per_window": n,
            "d2h_bytes_per_batch": B * 196608}


def config5_leg(dev, B, steps, warmup, n_ident=4, nstreams=1):
    """BASELINE config 5 on one GPU: linknet/3, every batch mixes 4 source identities (per-sample
    identity rows into the AAD identity path, dp.swap_mixed_identities); per GPU of the 8-GPU config."""
    from ghost_amd.inference.dp import swap_mixed_identities
    G = make_model("linknet", 3, torch.bfloat16, dev)
    crops = torch.from_numpy(np.random.Generator(np.random.PCG64(77)).integers(0, 256, size=(B, 256, 256, 3),
                                                                            dtype=np.uint8)).to(dev)
    zs = identity_rows(n_ident, dev)
    idx = (torch.arange(B, device=dev) % n_ident).to(torch.int32)
    table = G.identity_table(zs)               # the 4 identities' projections once per video
    ns = max(1, nstreams)
    outs = [torch.empty(B, 256, 256, 3, dtype=torch.uint8, device=dev) for _ in range(ns)]
    main = torch.cuda.current_stream(dev)
    comp = compute_streams(dev, ns)
    for c in comp[1:]:
        c.wait_stream(main)
    k = [0]

    def step():   # batch k on compute stream k % ns (ns batches in flight, as the headline loop)
        i = k[0] % ns
        with torch.cuda.stream(comp[i]):
            swap_mixed_identities(crops, idx, zs, G, out=outs[i], table=table)
        k[0] += 1

    el = timed(step, steps, warmup)
    del G
    torch.cuda.empty_cache()
    return {"workload": f"config 5 per GPU: batch={B} crops mixing {n_ident} identities, AEI_Net linknet "
                        f"num_blocks=3 bf16, u8 in -> u8 out, {ns} batch(es) in flight",
            "frames_per_s": round(B * steps / el, 1),
            "ms_per_batch": round(el * 1e3 / steps, 3)}


def config5_multi_leg(dev, world, frames_per_gpu=120, n_ident=4, BS=64, reps=3, G=None, crop=224):
    """BASELINE config 5 as one pipeline on every rank (N = 1..8): a synthetic video of frames_per_gpu * N frames
    with n_ident target identities (each present in ~90 % of the frames), per identity its crop_frames (224x224
    uint8 crops or []) and a source embedding; ``dp.model_inference_multi`` (core.py:56-88 over all identities at
    once): resize_frames on the device, the identities' present crops as one sequence sharded contiguously over
    the ranks, mixed-identity batches (per-sample embedding rows) with two in flight, each batch gathered to rank 0
    (RCCL gather at N > 1), rank 0 assembling final_frames_list.  Timed: ``reps`` calls after one warm-up, each
    bracketed by a barrier + device sync, max over ranks; output 'device' (rank 0 holds the swapped crops in HBM)
    and 'host' (rank 0 also copies them to pinned host memory, overlapped per batch).  ``G`` / ``crop``: a stand-in
    swap and 256-px crops for the gloo test of the N > 1 reporting (tests/test_dp_cpu.py)."""
    from ghost_amd.inference.dp import model_inference_multi
    own = G is None
    if own:
        G = make_model("linknet", 3, torch.bfloat16, dev)
    nf = frames_per_gpu * world
    rng = np.random.Generator(np.random.PCG64(55))
    pool = rng.integers(0, 256, size=(48, crop, crop, 3), dtype=np.uint8)    # distinct crops, reused by reference
    present = rng.random((n_ident, nf)) > 0.1
    embeds = identity_rows(n_ident, torch.device("cpu"))
    idents = []
    for q in range(n_ident):
        cf = [pool[(q * 7 + i) % len(pool)] if present[q, i] else [] for i in range(nf)]
        idents.append((cf, embeds[q:q + 1]))
    n_crops = int(present.sum())
    out = {"workload": f"config 5 as one pipeline: {nf}-frame video ({frames_per_gpu} per GPU), {n_ident} identities, "
                       f"{n_crops} face crops (224x224 crop_frames -> device resize_frames -> mixed-identity "
                       f"linknet/3 bf16 batches of {BS}, two in flight, sharded over {world} GPU(s), gathered to "
                       "rank 0 -> final_frames_list)", "crops": n_crops, "frames": nf}
    for mode in ("device", "host"):
        res = model_inference_multi(idents, G, BS=BS, device=dev, collect="rank0", output=mode)   # warm-up
        del res
        ts = []
        for _ in range(reps):
            if world > 1:
                dist.barrier()
            device_sync(dev)
            t0 = time.perf_counter()
            res = model_inference_multi(idents, G, BS=BS, device=dev, collect="rank0", output=mode)
            device_sync(dev)
            if world > 1:
                dist.barrier()
            ts.append(time.perf_counter() - t0)
            if res is not None:
                assert len(res) == n_ident and all(len(r) == nf for r in res)
            del res
        el = float(np.median(ts))
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        out[mode] = {"crops_per_s": round(n_crops / el, 1), "seconds": round(el, 4)}
    if own:
        del G
        torch.cuda.empty_cache()
    return out


def video_leg(G, dev, n_frames, BS=64, H=1080, W=1920):
    """BASELINE config 3 on one GPU, after host detection/alignment (models absent here: synthetic
    pre-aligned crops, affine transforms and masks).  Timed end to end:
      1. swap_identity_frames (core.py:57-88): H2D of the identity's crops, BS-batched swaps with a
         per-batch D2H of the uint8 result (overlapped), `present` re-insertion (5 % faceless frames);
      2. paste-back (get_final_video, video_processing.py:207-241): the full 1080p frames H2D in chunks,
         warp + mask composite on the device (blend.blend_swaps) from the device-resident swaps, D2H of
         the blended frames; copies on their own streams overlap the previous chunk's blend.
    The swap is resized 256 -> 224 as the reference does (cv2.resize INTER_LINEAR, on the device) before
    the warp; the masks (face_mask_static: hull fill, erode, border fade, Gaussian blur) are built on the
    device from per-frame landmarks; landmark detection and the video writer stay on the host."""
    from ghost_amd.inference.blend import blend_swaps
    from ghost_amd.inference.core import swap_identity_frames
    rng = np.random.Generator(np.random.PCG64(9))
    present = (rng.random(n_frames) > 0.05).astype(np.int64)
    n_face = int(present.sum())
    crops = rng.integers(0, 256, size=(n_face, 256, 256, 3), dtype=np.uint8)
    tile = torch.from_numpy(rng.integers(0, 256, size=(16, H, W, 3), dtype=np.uint8))
    frames_h = torch.empty(n_frames, H, W, 3, dtype=torch.uint8, pin_memory=True)
    for i in range(0, n_frames, 16):
        frames_h[i:i + 16] = tile[:min(16, n_frames - i)]
    # crop <- frame affine maps (a 224-px crop of a ~300 px face somewhere in the frame)
    ang = rng.uniform(-0.3, 0.3, n_frames)
    sc = rng.uniform(0.7, 0.9, n_frames)
    tx, ty = rng.uniform(600, 1300, n_frames), rng.uniform(200, 700, n_frames)
    mats = np.zeros((n_frames, 2, 3), np.float32)
    mats[:, 0, 0], mats[:, 0, 1] = sc * np.cos(ang), -sc * np.sin(ang)
    mats[:, 1, 0], mats[:, 1, 1] = sc * np.sin(ang), sc * np.cos(ang)
    mats[:, 0, 2] = -(mats[:, 0, 0] * tx + mats[:, 0, 1] * ty)
    mats[:, 1, 2] = -(mats[:, 1, 0] * tx + mats[:, 1, 1] * ty)
    # 106 landmarks per frame as the landmark model would return them on the 224 x 224 swap (synthetic: a jaw /
    # forehead contour + interior points, jittered per frame); face_mask_static's params from the first frame,
    # reused for the identity's later frames (video_processing.py:219-223)
    from ghost_amd.inference.masks import face_masks, mask_params
    t_ = np.linspace(0.15 * np.pi, 0.85 * np.pi, 33) + np.pi
    base = np.concatenate([np.stack([112 + 78 * np.cos(-t_), 118 + 92 * np.sin(-t_)], 1),
                           np.stack([112 + rng.uniform(-60, 60, 73), 118 + rng.uniform(-70, 60, 73)], 1)])
    lms = (base[None] + rng.normal(0, 1.5, (n_frames, 106, 2))).astype(np.float32)
    lm_tgt = (base + rng.normal(0, 1.5, (106, 2))).astype(np.float32)
    params = np.tile(np.array(mask_params(lms[0], lm_tgt), np.int32), (n_frames, 1))
    masks_d = torch.empty(n_frames, 224, 224, dtype=torch.float32, device=dev)
    mats_d = torch.from_numpy(mats).to(dev)
    valid_d = torch.from_numpy(present.astype(np.int32)).to(dev)
    z = identity_rows(1, dev)
    CH = 32
    bufs = [torch.empty(CH, H, W, 3, dtype=torch.uint8, device=dev) for _ in range(2)]
    s_in, s_out = stream_set(dev).h2d, stream_set(dev).d2h
    cur = torch.cuda.current_stream(dev)

    ev_times = {"masks": [], "blend": []}

    def bracket(kind):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev_times[kind].append((e0, e1))
        return e0, e1

    def run():
        for v in ev_times.values():
            v.clear()
        e0, e1 = bracket("masks")
        e0.record(cur)
        face_masks(lms, params, 224, 224, dev, out=masks_d)      # face_mask_static for every frame, on the GPU
        e1.record(cur)
        final, swaps_d = swap_identity_frames(crops, present, z, G, BS=BS, device=dev, return_device=True)
        # frame-indexed device swaps (faceless frames: a zero row, masked off by valid)
        idx = torch.from_numpy(np.maximum(np.cumsum(present) - 1, 0)).to(dev)
        swaps_f = swaps_d.index_select(0, idx)
        freed = [None, None]
        for c, f0 in enumerate(range(0, n_frames, CH)):
            f1 = min(n_frames, f0 + CH)
            b = bufs[c % 2]
            with torch.cuda.stream(s_in):
                if freed[c % 2] is not None:
                    s_in.wait_event(freed[c % 2])
                b[:f1 - f0].copy_(frames_h[f0:f1], non_blocking=True)
                loaded = torch.cuda.Event()
                loaded.record(s_in)
            cur.wait_event(loaded)
            e0, e1 = bracket("blend")
            e0.record(cur)
            blend_swaps(b[:f1 - f0], swaps_f[f0:f1], masks_d[f0:f1], mats_d[f0:f1], valid_d[f0:f1], resize_to=224)
            e1.record(cur)
            blended = torch.cuda.Event()
            blended.record(cur)
            with torch.cuda.stream(s_out):
                s_out.wait_event(blended)
                frames_h[f0:f1].copy_(b[:f1 - f0], non_blocking=True)   # result_frames[i] = final
                ev = torch.cuda.Event()
                ev.record(s_out)
                freed[c % 2] = ev
        s_out.synchronize()
        return final

    run()                                   # warm-up (allocations, first launches)
    torch.cuda.synchronize()
    els = []
    for _ in range(3):                      # three timed passes over the video, median reported
        t0 = time.perf_counter()
        final = run()
        torch.cuda.synchronize()
        els.append(time.perf_counter() - t0)
    el = float(np.median(els))
    assert len(final) == n_frames and sum(1 for f in final if len(f)) == n_face
    return {"workload": f"config 3: {n_frames}-frame {W}x{H} video, 1 identity, {n_face} frames with a face; "
                        f"crops H2D -> swaps (BS={BS}, per-batch D2H) -> present re-insertion -> frames H2D -> "
                        "device face masks (face_mask_static from per-frame landmarks) + resize 256->224 + "
                        "paste-back -> frames D2H (host detection/alignment/landmark model/writer excluded)",
            "frames_per_s": round(n_frames / el, 1), "seconds": round(el, 3),
            "passes_frames_per_s": [round(n_frames / e, 1) for e in els],
            "host_bytes_moved": int(n_face * 196608 * 2 + 2 * n_frames * H * W * 3),
            # device time of the paste-back pieces (HIP events on the compute stream, recorded after the wait for each
            # chunk's H2D copy; the blend brackets include the 256 -> 224 resize)
            "device_ms": {k: round(sum(a.elapsed_time(b) for a, b in v), 3) for k, v in ev_times.items()}}


def latency_leg(dev, n=20):
    """BASELINE config 1 on the GPU: one 256x256 image-to-image swap (B = 1, unet/2), fp32 and bf16.
    latency_ms = wall time of one synchronous swap_u8 call (median of n, after warm-up); host_ms = the
    host time of the call alone (the Python wrapper + the native plan's launches onto an idle stream,
    median of n); graphed = the same through GraphedSwap (one HIP graph launch per call)."""
    out = {"workload": "config 1 on 1 GPU: B=1 unet/2 swap_u8 (u8 crop in -> u8 swap out, device-resident), "
                       "one call at a time, synchronised after each"}
    crop = torch.from_numpy(np.random.Generator(np.random.PCG64(21)).integers(0, 256, (1, 256, 256, 3),
                                                                           dtype=np.uint8)).to(dev)
    z = identity_rows(1, dev)
    for name, dt in (("fp32", torch.float32), ("bf16", torch.bfloat16)):
        G = make_model("unet", 2, dt, dev)
        y = torch.empty(1, 256, 256, 3, dtype=torch.uint8, device=dev)
        for _ in range(5):
            G.swap_u8(crop, z, out=y)
        torch.cuda.synchronize()
        lat, host = [], []
        for _ in range(n):
            t0 = time.perf_counter()
            G.swap_u8(crop, z, out=y)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            host.append(t1 - t0)
            lat.append(t2 - t0)
        out[name] = {"latency_ms": round(float(np.median(lat)) * 1e3, 3),
                     "host_ms": round(float(np.median(host)) * 1e3, 3)}
        # the same swap with the source identity's projections prepared once (AEI_Net.identity_table: inference.py
        # embeds the source once and swaps it into every target image), one gather instead of the two GEMMs
        table = G.identity_table(z)
        idx = torch.zeros(1, dtype=torch.int32, device=dev)
        for _ in range(3):
            G.swap_u8_indexed(crop, table, idx, out=y)
        torch.cuda.synchronize()
        lat = []
        for _ in range(n):
            t0 = time.perf_counter()
            G.swap_u8_indexed(crop, table, idx, out=y)
            torch.cuda.synchronize()
            lat.append(time.perf_counter() - t0)
        out[name]["identity_table_latency_ms"] = round(float(np.median(lat)) * 1e3, 3)
        # the same swap replayed as one HIP graph (ghost_amd.inference.GraphedSwap: inputs copied into the
        # captured buffers, one hipGraphLaunch; identical bytes); at B = 1 the plan is one chain of kernels
        # whatever two_streams says (batches under 8 frames run on one stream), so one capture is timed
        from ghost_amd.inference import GraphedSwap
        for key, ts in (("graphed", 0),):
            gs = GraphedSwap(G, 1, dev, two_streams=ts)
            for _ in range(5):
                gs(crop, z, out=y)
            torch.cuda.synchronize()
            lat, host = [], []
            for _ in range(n):
                t0 = time.perf_counter()
                gs(crop, z, out=y)
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                host.append(t1 - t0)
                lat.append(t2 - t0)
            out[name][key] = {"latency_ms": round(float(np.median(lat)) * 1e3, 3),
                              "host_ms": round(float(np.median(host)) * 1e3, 3)}
            del gs
        # eager with one stream (the plan option two_streams = 0)
        G.set_option("two_streams", 0)
        for _ in range(3):
            G.swap_u8(crop, z, out=y)
        torch.cuda.synchronize()
        lat = []
        for _ in range(n):
            t0 = time.perf_counter()
            G.swap_u8(crop, z, out=y)
            torch.cuda.synchronize()
            lat.append(time.perf_counter() - t0)
        out[name]["one_stream_latency_ms"] = round(float(np.median(lat)) * 1e3, 3)
        del G
        torch.cuda.empty_cache()
    return out


def host_cpu_budget():
    """CPUs this process may use: the cgroup quota when one is set (the GPU box gives a job a share
    of a large host, whose os.cpu_count() is many times that share), else the affinity mask."""
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(backbone, nb, batches):
    """Oracle (CPU fp32 restatement, same ATen op sequence as the reference) frames/s on this host:
    BASELINE.md §4 — B in {1, 64}, 1 warm-up + 3 timed iterations each, time.perf_counter."""
    from oracle import aei_ref
    threads = host_cpu_budget()
    torch.set_num_threads(threads)
    p = aei_ref.make_weights(aei_ref.param_specs(backbone, nb))
    per_b = {}
    for bs in batches:
        xt, z = aei_ref.make_inputs(bs, seed=3)
        aei_ref.aei_forward(p, xt, z, backbone, nb)        # warm-up
        t0 = time.perf_counter()
        for _ in range(3):
            aei_ref.aei_forward(p, xt, z, backbone, nb)
        el = time.perf_counter() - t0
        per_b[str(bs)] = {"frames_per_s": round(3 * bs / el, 3), "s_per_batch": round(el / 3, 3)}
    best = max(batches)
    return {"value": per_b[str(best)]["frames_per_s"], "unit": "frames/s", "cores": threads, "kind": "port",
            "os_cpu_count": os.cpu_count(), "by_batch": per_b,
            "sample": f"{backbone}/{nb} fp32 (oracle/aei_ref.py) at B in {list(batches)}: 1 warm-up + 3 timed "
                      f"iterations each on {threads} threads (the process's CPU quota); value = B={best}"}


def device_sync(dev: torch.device) -> None:
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def timed_region(step, drain, steps, warmup, world, dev, before_timed=None, per_rank=None) -> float:
    """W untimed warm-up steps, then EXACTLY K timed steps bracketed by a barrier + device synchronize on
    both sides (every step's collective drained inside the region); returns the max over ranks of the
    K steps' wall time (an all-gather of every rank's time over the group: RCCL on the GPU, gloo in the CPU
    test).  per_rank: a list that receives every rank's own time, in rank order."""
    for _ in range(warmup):
        step()
    drain()
    device_sync(dev)
    if before_timed is not None:
        before_timed()
    if world > 1:
        dist.barrier()
    device_sync(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    drain()
    device_sync(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    times = [el]
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        ts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(ts, t)
        times = [float(x.item()) for x in ts]
        el = max(times)
    if per_rank is not None:
        per_rank[:] = times
    return el


def headline_record(world, B, steps, warmup, el, backbone, num_blocks, identities, dtype, nstreams,
                    per_rank=None) -> dict:
    """The JSON line's headline fields: value = frames of ALL ranks / max-over-ranks time (weak scaling,
    B frames per GPU per step).  rccl_world = the process group's own size (dist.get_world_size(), 1 without a
    group), per_rank_s = every rank's timed region."""
    frames = world * B * steps
    cfg = "config 5 (mixed identities)" if identities > 1 else ("config 4" if world > 1 else "config 2")
    return {
        "metric": BASELINE_METRIC,
        "value": round(frames / el, 2), "unit": "frames/s", "n_gpus": world, "steps": steps, "warmup": warmup,
        "ms_per_step": round(el / steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": dtype if dtype == "fp32" else "bf16", "data": "synthetic",
        "config": {"workload": f"BASELINE {cfg}: batch={B} synthetic 256x256 aligned faces per GPU"
                               + (f" mixing {identities} identities" if identities > 1 else "")
                               + f", AEI_Net {backbone} num_blocks={num_blocks}, faceshifter_batch "
                                 "(u8 in -> u8 out, device-resident; D2H in legs.d2h)"
                               + (", RCCL all-gather of swapped crops" if world > 1 else ""),
                   "global_batch": world * B, "per_gpu_batch": B, "backbone": backbone,
                   "num_blocks": num_blocks, "identities": max(1, identities),
                   "parallelism": f"dp{world}", "batches_in_flight": nstreams,
                   "identity_projection": "fc1/fc2/up1 once per source identity (AEI_Net.identity_table, before the "
                                          "timed region), gathered per sample by identity index in every step; "
                                          "legs.per_batch_projection: the literal per-batch projection"},
        "rccl_world": dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1,
        "per_rank_s": [round(t, 6) for t in (per_rank or [el])],
    }


def launch_ranks(a, argv) -> int:
    """``--gpus N`` (N > 1) with no outside launcher (no WORLD_SIZE in the environment): start N ranks of this same
    command as child processes (subprocess.Popen, never exec; this process makes no GPU call at all), one per GPU,
    with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set as torch.distributed.run sets
    them.  Rank 0's stdout (the JSON line) is relayed line by line as it arrives; the other ranks' stdout goes to
    stderr.  The first rank to fail ends the others (their exact PIDs); returns non-zero if any rank failed or
    rank 0 printed no JSON line with n_gpus == N.  The reference's loop it spreads: utils/inference/core.py:72-74."""
    import socket
    import subprocess
    import threading
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    me = os.path.abspath(__file__)
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", me] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno(), text=True))
    lines = []

    def relay():
        for ln in procs[0].stdout:
            sys.stdout.write(ln)
            sys.stdout.flush()
            lines.append(ln)
    th = threading.Thread(target=relay, daemon=True)
    th.start()
    rc = 0
    while any(p.poll() is None for p in procs):
        bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
        if bad:
            rc = bad[0]
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        time.sleep(0.2)
    th.join(timeout=10)
    if rc == 0:
        rc = next((p.returncode for p in procs if p.returncode), 0)
    if rc:
        print(f"bench.py: a rank exited with status {rc}", file=sys.stderr)
        return rc if rc > 0 else 1
    recs = []
    for ln in lines:
        try:
            recs.append(json.loads(ln))
        except ValueError:
            pass
    if not any(isinstance(x, dict) and x.get("n_gpus") == a.gpus for x in recs):
        print(f"bench.py: rank 0 printed no JSON line with n_gpus = {a.gpus}", file=sys.stderr)
        return 1
    return 0


def standin_main(a, world, rank):
    """The launcher path on the CPU (tests/test_dp_cpu.py): gloo ranks, a deterministic stand-in for the swap on
    small crops, GatherPipeline + timed_region + headline_record as the GPU run uses them."""
    from ghost_amd.inference.dp import GatherPipeline
    dev = torch.device("cpu")
    if world > 1:
        dist.init_process_group("gloo")
    B = a.batch

    def swap(c, o):
        o.copy_((255 - c).flip(-1))
    pipe = GatherPipeline(swap, (B, 4, 4, 3), dev, depth=2)
    crops = torch.full((B, 4, 4, 3), rank, dtype=torch.uint8)
    per = []
    el = timed_region(lambda: pipe.submit(crops), pipe.drain, a.steps, a.warmup, world, dev, per_rank=per)
    if rank == 0:
        res = headline_record(world, B, a.steps, a.warmup, el, a.backbone, a.num_blocks, a.identities, a.dtype, 1, per)
        res["data"] = "synthetic (CPU stand-in swap, gloo)"
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        return launch_ranks(a, argv)             # N ranks of this command, no GPU call in this process
    world = int(env_world or "1")
    if env_world is not None and a.gpus != world:
        print(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if a.standin_cpu:
        standin_main(a, world, rank)
        return 0
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    stream_set(dev)       # the process's streams first, so they hold distinct hardware queues (streams.py)

    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    G = make_model(a.backbone, a.num_blocks, dt, dev)
    for kv in a.opt:
        name, val = kv.split("=")
        G.set_option(name, int(val))

    B = a.batch
    rng = np.random.Generator(np.random.PCG64(1000 + rank))
    crops = torch.from_numpy(rng.integers(0, 256, size=(B, 256, 256, 3), dtype=np.uint8)).to(dev)
    zs = identity_rows(max(1, a.identities), dev)
    z = zs[:1]
    # the source identities' projections (every AADLayer's fc1/fc2 and up1) once, before the timed region — once per
    # identity per video, as a weight pack is once per model; each step gathers its samples' rows by identity index
    # (config 5: mixed identities in every batch; config 2: one identity, an all-zero index)
    table = G.identity_table(zs)
    idx = (torch.arange(B, device=dev) % max(1, a.identities)).to(torch.int32)

    def swap(c, o):
        return G.swap_u8_indexed(c, table, idx, out=o)
    # swap -> all-gather of the uint8 swaps to every rank; the gather of step k overlaps step k + 1
    # (dp.GatherPipeline; GHOST_DP_OVERLAP=0 gathers synchronously after each step).  --streams 2 (default)
    # keeps two independent batches in flight on two HIP streams: one batch's latency-bound low-resolution
    # stages overlap the other's HBM/MFMA-bound stages (every batch still runs its whole forward)
    from ghost_amd.inference.dp import GatherPipeline
    pipe = GatherPipeline(swap, (B, 256, 256, 3), dev,
                          depth=2 if os.environ.get("GHOST_DP_OVERLAP", "1") != "0" else 1,
                          streams=max(1, a.streams))

    def step():
        slot = pipe.submit(crops)
        if pipe.depth == 1:
            pipe.result(slot)

    prof = not a.no_profile
    names = ["aad_all", "aad_dual_256", "conv3x3_all", "conv3x3_256", "in_stats_mask", "encoder", "upsample",
             "id_proj"]
    classes = {}

    def before_timed():
        if prof:
            # inside the timed region only the roofline kernel is bracketed (one HIP event pair per step,
            # recorded on the launch stream around each of its launches)
            G.profile(1 << names.index("aad_dual_256"))

    per_rank = []
    el = timed_region(step, pipe.drain, a.steps, a.warmup, world, dev, before_timed, per_rank)
    iso = {}
    clock = {"timed": (0.0, 0), "isolated": (0.0, 0)}
    if prof:
        classes["aad_dual_256"] = G.profile_read(names.index("aad_dual_256"))
        clock["timed"] = G.profile_clock()
        # per-class breakdown from a separate, untimed pass with one batch at a time (every kernel class
        # bracketed; with batches in flight a class's time would include the other batch's kernels)
        pipe.drain()
        pipe1 = GatherPipeline(swap, (B, 256, 256, 3), dev, depth=pipe.depth,
                               streams=1)
        G.profile(0xFF)
        for _ in range(a.steps):
            pipe1.submit(crops)
        pipe1.drain()
        torch.cuda.synchronize()
        for i, n in enumerate(names):
            if n != "aad_dual_256":
                classes[n] = G.profile_read(i)
            else:
                iso = G.profile_read(i)
        clock["isolated"] = G.profile_clock()
        G.profile(0)

    # legs every rank runs (N >= 1): config 5 as one multi-identity pipeline, gathered to rank 0
    multi_legs = {}
    if "config5_multi" in [s for s in a.legs.split(",") if s] and a.c5_frames > 0:
        pipe.drain()
        multi_legs["config5_multi"] = config5_multi_leg(dev, world, a.c5_frames)
    if rank == 0:
        res = headline_record(world, B, a.steps, a.warmup, el, a.backbone, a.num_blocks, a.identities, a.dtype,
                              pipe.nstreams, per_rank)
        if prof and classes["aad_dual_256"]["launches"]:
            c = classes["aad_dual_256"]
            per_launch_formula = c["bytes"] / c["launches"]
            ev_s = c["ms"] / c["launches"] / 1e3                 # HIP-event bracket (includes queueing)
            clk_us, clk_n = clock["timed"]
            ca8 = 32 if a.backbone == "linknet" else 64     # z_attr8 channels (AEI_Net.py:110,118)
            # layers in the kernel: the formula bytes per launch are L * B*256^2*(2*64 + Ca)*2
            nl = max(1, round(per_launch_formula / (B * 65536 * (2 * 64 + ca8) * 2)))
            # minimum bytes of the fused kernel: h_in's 128x128 source once, z_attr8 once, nl outputs; an output
            # whose layer feeds AADBlk8's conv to 3 channels through tap partials (GHOST_AEI_OPT_TAP_PARTIALS) is
            # 15 fp16 row-summed partials per pixel instead of 64 bf16 channels: nb >= 2 -> last_add_block's layer (mode
            # 2); nb = 1 -> the h path's layer (modes 1, 2) and last_add_block's (mode 2)
            zp = G.get_option("tap_partials") if a.dtype == "bf16" else 0
            per_launch_min, n_part, zpm = aad_v4_min_bytes(B, ca8, nl, a.num_blocks, zp)
            v5 = G.kernel_variant("aad_dual_256") == "v5"
            # the launched instantiation (aad_v3.hip aad_v3_t): v5 <T, Ca, L, RELU, ZPM, ASMW = ZPM != 0>
            kname = (f"aad_v5_kernel<__bf16, {ca8}, {nl}, true, {zpm}, {'true' if zpm else 'false'}>" if v5
                     else f"aad_v4_kernel<{ca8}, {nl}, true, true, {zpm}>")
            # duration per launch: the committed rocprofv3 --kernel-trace --stats average of this exact symbol in the
            # timed configuration (profiles/rNN_kernel_stats.csv, written by tools/profile_round.sh from this bench
            # command) when the summary has its row — so every fraction below can be recomputed from profiles/ —
            # else the kernel's own live execution span (in-kernel clock: first workgroup start -> last wave end);
            # the live clock is always reported beside it (live_clock_us) with its ratio to the rocprof row
            clocked = clk_n > 0
            live_s = clk_us / clk_n / 1e6 if clocked else ev_s
            tr = pmc_traffic(kname)
            rp = rocprof_avg_us(kname)
            use_rp = bool(rp and rp.get("timed_avg_us"))
            per_launch_s = rp["timed_avg_us"] / 1e6 if use_rp else live_s
            ach = per_launch_min / per_launch_s / 1e9

            def fr(nbytes, t):
                return round(nbytes / t / 1e9 / HBM_PEAK_GBS, 4)
            res["roofline"] = {
                "kernel": f"{kname}: AADBlk8's block-input AAD kernel at 256x256, {nl} AADLayer(s) sharing h_in/"
                          "z_attr, h_in = bilinear x2 of the 128x128 block output sampled in-kernel (IN-normalise, "
                          "sigmoid mask, MFMA gamma/beta, blend, ReLU)"
                          + (f"; {n_part} layer(s) writing tap partials" if n_part else ""),
                "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4),
                "traffic": tr["bytes_per_launch"] if tr else None,
                "avg_launch_us": round(per_launch_s * 1e6, 2),
                "duration_source": (f"rocprofv3 kernel-trace average of this symbol in the timed configuration "
                                    f"({rp['timed_source']}, {rp['timed_calls']} calls)" if use_rp else
                                    "in-kernel wall clock (earliest workgroup start to latest wave end, s_memrealtime "
                                    "stamps) of every launch in the timed region" if clocked else
                                    "HIP events on the launch stream around each launch in the timed region"),
                "live_clock_us": round(live_s * 1e6, 2), "launches_timed": clk_n if clocked else c["launches"],
                "bytes_per_launch": per_launch_min,
                "bytes_note": "achieved = minimum bytes of the fused kernel (128x128 h_in source + z_attr8 + outputs "
                              "as stored: 64 bf16 channels, or 15 fp16 row-summed tap partials per pixel) / launch duration",
                "fractions": {
                    "minimum_bytes": fr(per_launch_min, per_launch_s),
                    "physical_pmc": fr(tr["bytes_per_launch"], per_launch_s) if tr else None,
                    "survey_8d_formula": fr(per_launch_formula, per_launch_s),
                    "formula_bytes_per_launch": per_launch_formula,
                    "pmc_source": tr["source"] if tr else None},
                "timed_region_latency": {
                    "avg_launch_us": round(ev_s * 1e6, 2), "launches": c["launches"],
                    "note": (f"HIP events on the launch stream; with {pipe.nstreams} batches in flight the bracket "
                             "includes queueing behind the other stream's kernels")},
                "rocprof": rp,
            }
            if tr:
                res["roofline"]["traffic_detail"] = tr
            # this run's own fraction (minimum bytes / the live in-kernel clock of the timed region), flagged when it
            # departs from the committed trace row by more than 10 %
            res["roofline"]["frac_live"] = fr(per_launch_min, live_s)
            if use_rp:
                ratio = live_s * 1e6 / rp["timed_avg_us"]
                res["roofline"]["live_clock_vs_rocprof"] = round(ratio, 3)
                res["roofline"]["live_departs_from_committed_row"] = bool(abs(ratio - 1.0) > 0.10)
            mp = mfma_profile(mangle(kname) or kname)
            if mp and mp.get("generator", {}).get("kernels"):
                res["roofline"]["issue_counters"] = mp["generator"]["kernels"][0] | {"source": mp["source"]}
            if iso.get("launches"):
                # the same kernel with one batch on the GPU (untimed pass): live in-kernel clock, and the
                # one-stream trace row (profiles/rNN_kernel_stats_1stream.csv) beside it
                iso_us, iso_n = clock["isolated"]
                iso_s = iso_us / iso_n / 1e6 if iso_n else iso["ms"] / iso["launches"] / 1e3
                rp_iso = rp.get("isolated_avg_us") if rp else None
                res["roofline"]["isolated"] = {
                    "avg_launch_us": round(iso_s * 1e6, 2), "achieved": round(per_launch_min / iso_s / 1e9, 1),
                    "frac": fr(per_launch_min, iso_s),
                    "formula_frac": fr(per_launch_formula, iso_s),
                    "physical_frac": fr(tr["bytes_per_launch"], iso_s) if tr else None,
                    "event_avg_launch_us": round(iso["ms"] / iso["launches"] * 1e3, 2),
                    "launches": iso["launches"],
                    "rocprof_avg_us": rp_iso,
                    "rocprof_frac": fr(per_launch_min, rp_iso / 1e6) if rp_iso else None,
                    "live_vs_rocprof": round(iso_s * 1e6 / rp_iso, 3) if rp_iso else None,
                    "note": "one batch at a time (untimed pass, in-kernel clock); rocprof_avg_us is the one-stream "
                            "trace row (rocprof.isolated_source)"}
            cc = classes["conv3x3_all"]
            if cc["launches"]:
                tf = cc["flops"] / (cc["ms"] / 1e3) / 1e12
                res["roofline_conv3x3"] = {"bound": "mfma", "achieved": round(tf, 1), "peak": BF16_PEAK_TFLOPS,
                                           "unit": "TFLOP/s", "frac": round(tf / BF16_PEAK_TFLOPS, 4)}
                mp = mfma_profile("conv3x3_halo")
                if mp and "generator" in mp:
                    # PMC MFMA utilisation of the halo 3x3 convs (committed rocprofv3 --pmc rows) and the whole step
                    res["roofline_conv3x3"]["mfma_counters"] = {
                        "source": mp["source"], "definition": mp["definition"],
                        "step_mfma_busy": mp["generator"]["totals"].get("mfma_busy"),
                        "kernels": mp["generator"]["kernels"]}
            aad = classes["aad_all"]
            if aad["ms"]:
                # SURVEY.md §8d definition: sum over AADLayers of |h_in|+|z_attr|+|out| / AAD kernel time
                res["aad_decoder_gbs"] = round(AAD_BYTES_PER_FRAME[a.backbone] * B * a.steps
                                               / (aad["ms"] / 1e3) / 1e9, 1)
                res["aad_decoder_hbm_frac"] = round(res["aad_decoder_gbs"] / HBM_PEAK_GBS, 4)
            res["kernel_ms_per_step"] = {k: round(v["ms"] / a.steps, 3) for k, v in classes.items()}
            res["kernel_ms_per_step_note"] = ("aad_dual_256 from the timed region; the other classes from an "
                                              "untimed one-batch-at-a-time pass with every class bracketed by "
                                              "HIP events")
        legs = [s for s in a.legs.split(",") if s] if world == 1 else []
        if legs or multi_legs:
            res["legs"] = dict(multi_legs)
        if "per_batch_projection" in legs:
            res["legs"]["per_batch_projection"] = per_batch_projection_leg(G, crops, zs, idx, a.steps, a.warmup,
                                                                           pipe.nstreams)
        if "d2h" in legs:
            res["legs"]["d2h"] = d2h_leg(swap, crops, a.steps, pipe.nstreams)
        if "fp16" in legs:
            res["legs"]["fp16"] = fp16_leg(dev, crops, z, a.steps, 3, a.backbone, a.num_blocks, pipe.nstreams)
        if "video" in legs and a.video > 0:
            res["legs"]["config3_video"] = video_leg(G, dev, a.video)
        if "config5" in legs:
            res["legs"]["config5"] = config5_leg(dev, B, a.steps, 3, nstreams=pipe.nstreams)
        if "latency" in legs:
            res["legs"]["config1_latency"] = latency_leg(dev)
        arc_batches = [int(b) for b in str(a.arc_batch).split(",") if b]
        if "arcface" in legs and arc_batches:
            # one batch at a time: two in flight measured neutral (the persistent 3x3 convs hold every CU)
            runs = [arcface_leg(dev, n, max(3, a.steps // 2), 1) for n in arc_batches]
            res["legs"]["arcface"] = dict(runs[0])
            res["legs"]["arcface"]["by_batch"] = {str(r["batch"]): {k: r[k] for k in ("ms_per_batch", "embeddings_per_s",
                                                                                     "mfma_frac")} for r in runs}
        batches = [int(b) for b in a.cpu_batches.split(",") if b]
        if world == 1 and batches:
            res["cpu_baseline"] = cpu_baseline(a.backbone, a.num_blocks, batches)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())

"""Per-stage bf16 parity of the MI355X throughput path against the bf16-storage-emulating oracle.

    python tools/bf16_bisect.py [--backbone unet --num-blocks 2 --batch 64 --rows 0,21,42,63] [--json out.json]

Runs AEI_Net bf16 at the full batch on the GPU (forward_taps: encoder maps, AADBlk1..7 outputs, Y),
the oracle (oracle/aei_ref.aei_forward_bf16_storage) on the sampled rows on the CPU, and prints
per-stage error figures; then the uint8 swap against the oracle's u8 frame (LSB histogram), and the
errors of the plain fp32 oracle / an fp16 evaluation (the reference's GPU precision) for scale.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import aei_ref  # noqa: E402


def stats(got, ref):
    d = (got.float() - ref.float()).abs()
    scale = float(ref.abs().mean()) or 1.0
    flat = d.flatten()
    if flat.numel() > (1 << 22):
        flat = flat[torch.randperm(flat.numel(), generator=torch.Generator().manual_seed(0))[:1 << 22]]
    return {"mean": float(d.mean()), "rel_mean": float(d.mean()) / scale, "max": float(d.max()),
            "p999": float(torch.quantile(flat, 0.999)), "ref_mean_abs": scale}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backbone", default="unet")
    ap.add_argument("--num-blocks", type=int, default=2)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--rows", default="0,21,42,63")
    ap.add_argument("--json", default=None)
    ap.add_argument("--fp16", action="store_true", help="also evaluate the fp16 restatement (slow on CPU)")
    a = ap.parse_args()
    from ghost_amd.network import AEI_Net
    dev = torch.device("cuda:0")
    bb, nb, B = a.backbone, a.num_blocks, a.batch
    rows = [int(r) for r in a.rows.split(",") if int(r) < B]
    p = aei_ref.make_weights(aei_ref.param_specs(bb, nb))
    G = AEI_Net(bb, num_blocks=nb, c_id=512, compute_dtype=torch.bfloat16).eval()
    G.load_state_dict(p)
    G = G.to(dev)
    xt, z = aei_ref.make_inputs(B, 11)
    U8 = torch.empty(B, 256, 256, 3, dtype=torch.uint8, device=dev)
    Y, attr, blocks = G.forward_taps(xt.to(dev), z.to(dev), out_u8=U8)
    torch.cuda.synchronize()
    t0 = time.time()
    ri = torch.tensor(rows)
    Ye, attr_e, blocks_e, t_e = aei_ref.aei_forward_bf16_storage(p, xt[ri], z[ri], bb, nb)
    t_oracle = time.time() - t0
    out = {"backbone": bb, "num_blocks": nb, "batch": B, "rows": rows, "oracle_s": round(t_oracle, 1), "stages": {}}
    for i, (g, r) in enumerate(zip(attr, attr_e), 1):
        out["stages"][f"z_attr{i}"] = stats(g[ri].cpu(), r)
    for k, (g, r) in enumerate(zip(blocks, blocks_e[:7]), 1):
        out["stages"][f"AADBlk{k}"] = stats(g[ri].cpu(), r)
    out["stages"]["Y"] = stats(Y[ri].cpu(), Ye)
    # isolated stages: each block fed the GPU's own stored input (previous block output, z_attr)
    ga = [a[ri].float().cpu() for a in attr]
    gb = [b[ri].float().cpu() for b in blocks]
    zr = z[ri]
    out["isolated"] = {}
    prev = aei_ref.up1_bf16_storage(zr, p)
    for k in range(1, 9):
        yk = aei_ref.gen_block_bf16_storage(prev, ga[k - 1], zr, p, bb, nb, k)
        if k < 8:
            out["isolated"][f"AADBlk{k}"] = stats(gb[k - 1], yk)
            prev = gb[k - 1]
        else:
            t8 = torch.tanh(yk)
            out["isolated"]["Y"] = stats(Y[ri].float().cpu(), aei_ref._q(t8))
            Ui = aei_ref.y_to_u8_bgr(t8)
            di = np.abs(U8[ri].cpu().numpy().astype(np.int16) - Ui.astype(np.int16))
            out["isolated"]["u8"] = {"max_lsb": int(di.max()), "mean_lsb": float(di.mean()),
                                     "hist_0_16plus": [int(h) for h in np.bincount(np.minimum(di.ravel(), 16),
                                                                                   minlength=17)]}
    # intrinsic bf16 error (emulation vs the fp32 oracle) and the fp16 reference precision
    y32, _ = aei_ref.aei_forward(p, xt[ri], z[ri], bb, nb)
    out["emulation_vs_fp32"] = stats(Ye, y32)
    out["gpu_vs_fp32"] = stats(Y[ri].cpu(), y32)
    if a.fp16:
        out["fp16_vs_fp32"] = stats(aei_ref.fp16_reference_forward(p, xt[ri], z[ri], bb, nb), y32)
    # uint8 swap path: u8 crops, one identity; u8 from the oracle's fp32 tanh (as the kernel does)
    crops = aei_ref.make_u8_crops(B, 4)
    U = G.swap_u8(torch.from_numpy(crops).to(dev), z[:1].to(dev)).cpu().numpy()
    tgt = aei_ref.transform_target(crops[rows])
    _, _, _, t_u = aei_ref.aei_forward_bf16_storage(p, tgt, torch.cat([z[:1]] * len(rows)), bb, nb)
    Ue = aei_ref.y_to_u8_bgr(t_u)
    du = np.abs(U[rows].astype(np.int16) - Ue.astype(np.int16))
    hist = np.bincount(np.minimum(du.ravel(), 16), minlength=17)
    out["u8_vs_emulation"] = {"max_lsb": int(du.max()), "mean_lsb": float(du.mean()),
                              "hist_0_16plus": [int(h) for h in hist], "frac_nonzero": float((du > 0).mean())}
    u32 = aei_ref.y_to_u8_bgr(aei_ref.aei_forward(p, tgt, torch.cat([z[:1]] * len(rows)), bb, nb)[0])
    d32 = np.abs(U[rows].astype(np.int16) - u32.astype(np.int16))
    out["u8_vs_fp32"] = {"max_lsb": int(d32.max()), "mean_lsb": float(d32.mean()),
                         "hist_0_16plus": [int(h) for h in np.bincount(np.minimum(d32.ravel(), 16), minlength=17)]}
    print(f"{bb}/{nb} B={B} rows={rows} (oracle {t_oracle:.1f}s)")
    print(f"{'stage':10s} {'mean':>10s} {'rel_mean':>10s} {'p999':>10s} {'max':>10s}")
    for k, v in out["stages"].items():
        print(f"{k:10s} {v['mean']:10.2e} {v['rel_mean']:10.2e} {v['p999']:10.2e} {v['max']:10.2e}")
    print("isolated (each block from the GPU's stored inputs):")
    for k, v in out["isolated"].items():
        if k != "u8":
            print(f"{k:10s} {v['mean']:10.2e} {v['rel_mean']:10.2e} {v['p999']:10.2e} {v['max']:10.2e}")
    print("isolated u8:", out["isolated"]["u8"])
    for k in ("emulation_vs_fp32", "gpu_vs_fp32", "fp16_vs_fp32"):
        if k in out:
            v = out[k]
            print(f"{k:18s} mean {v['mean']:.2e} p999 {v['p999']:.2e} max {v['max']:.2e}")
    print("u8 vs emulation:", out["u8_vs_emulation"])
    print("u8 vs fp32:", out["u8_vs_fp32"])
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

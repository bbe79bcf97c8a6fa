"""Where does a 16-bit AADBlk_k differ from its storage emulation?  (GPU box.)

    python tools/fp16_probe.py [--st fp16] [--block 7] [--batch 64]

Runs AEI_Net at the given storage dtype (forward_taps), then AADBlk_k from the GPU's own stored inputs
three ways on the CPU: the oracle's emulation (fp32 arithmetic), the same emulation in fp64 arithmetic
(same storage rounding points), and the fp64 emulation with the runtime's folded mask logit
(sum_c (wh_c rs_c) h_c + (bh - sum_c wh_c mu_c rs_c), aad_v3.hip).  Prints the error of each against
the GPU in units of the element's own ulp and of 2 ulp(max |ref|), the test's gate."""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import aei_ref as R  # noqa: E402

MANT = {"bf16": 7, "fp16": 10}
STORE = {"bf16": torch.bfloat16, "fp16": torch.float16}


def ulp_el(t, st):
    e = torch.floor(torch.log2(t.abs().double().clamp_min(2.0 ** -14)))
    return 2.0 ** (e - MANT[st])


def block64(y_prev, za, z_id, p, k, st, folded=False, nb=2):
    """AADBlk_k (cin != cout, unet) in fp64 arithmetic with the runtime's storage rounding points."""
    S = STORE[st]
    q = lambda t: t.to(S).double()   # noqa: E731
    pd = {kk: v.double() for kk, v in p.items() if kk.startswith(f"generator.AADBlk{k}.")}
    pre = f"generator.AADBlk{k}"
    za, z_id = za.double(), z_id.double().reshape(z_id.shape[0], -1)
    u = F.interpolate(y_prev.double(), scale_factor=2, mode="bilinear", align_corners=True)
    m = q(u)
    var, mean = torch.var_mean(u, dim=(2, 3), unbiased=False, keepdim=True)
    st_m = (mean, torch.rsqrt(var + R.IN_EPS))

    def aad(h_in, prefix, stats=None):
        mean, rstd = stats if stats is not None else (lambda v, mu: (mu, torch.rsqrt(v + R.IN_EPS)))(
            *torch.var_mean(h_in, dim=(2, 3), unbiased=False, keepdim=True))
        h = (h_in - mean) * rstd
        ga = F.conv2d(za, q(pd[f"{prefix}.conv1.weight"]), pd[f"{prefix}.conv1.bias"])
        ba = F.conv2d(za, q(pd[f"{prefix}.conv2.weight"]), pd[f"{prefix}.conv2.bias"])
        gi = F.linear(z_id, pd[f"{prefix}.fc1.weight"], pd[f"{prefix}.fc1.bias"])
        bi = F.linear(z_id, pd[f"{prefix}.fc2.weight"], pd[f"{prefix}.fc2.bias"])
        c = h.shape[1]
        A = ga * h + ba
        I = gi.reshape(-1, c, 1, 1) * h + bi.reshape(-1, c, 1, 1)
        wh, bh = pd[f"{prefix}.conv_h.weight"], pd[f"{prefix}.conv_h.bias"]
        if folded:   # the kernel's form, each term in fp32
            cf = (wh.reshape(1, c, 1, 1) * rstd).float()
            kk = (wh.reshape(1, c, 1, 1) * (-mean * rstd)).float().sum(1, keepdim=True)
            logit = (cf * h_in.float()).sum(1, keepdim=True) + kk + bh.float().reshape(1, 1, 1, 1)
            M = torch.sigmoid(logit.double())
        else:
            M = torch.sigmoid(F.conv2d(h, wh, bh))
        return q(F.relu((1 - M) * A + M * I))

    x = m
    for i in range(nb):
        a = aad(x, f"{pre}.add_blocks.{3 * i}", st_m if i == 0 else None)
        x = F.conv2d(a, q(pd[f"{pre}.add_blocks.{3 * i + 2}.weight"]), None, padding=1)
        if i < nb - 1:
            x = q(x)
    a = aad(m, f"{pre}.last_add_block.0", st_m)
    y = x + F.conv2d(a, q(pd[f"{pre}.last_add_block.2.weight"]), None, padding=1)
    return q(y)


def report(name, g, r, st):
    d = (g.double() - r.double()).abs()
    ue = d / ulp_el(r, st)
    gate = 2 * 2.0 ** (np.floor(np.log2(float(r.abs().max()))) - MANT[st])
    idx = int(d.argmax())
    print(f"{name:28s} max {float(d.max()):.3e} ({float(d.max()) / gate:.2f} gate) mean {float(d.mean()):.3e} "
          f"elem-ulp: >1 {int((ue > 1).sum())} >2 {int((ue > 2).sum())} max {float(ue.max()):.1f}; "
          f"argmax {np.unravel_index(idx, tuple(d.shape))} ref {float(r.flatten()[idx]):.4f} "
          f"gpu {float(g.flatten()[idx]):.4f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--st", default="fp16")
    ap.add_argument("--block", type=int, default=7)
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    from ghost_amd.network import AEI_Net
    dev = torch.device("cuda:0")
    p = R.make_weights(R.param_specs("unet", 2))
    if a.st == "fp16":
        G = AEI_Net("unet", num_blocks=2, c_id=512).eval()
        G.load_state_dict(p)
        G = G.to(dev).half()
    else:
        G = AEI_Net("unet", num_blocks=2, c_id=512, compute_dtype=torch.bfloat16).eval()
        G.load_state_dict(p)
        G = G.to(dev)
    xt, z = R.make_inputs(a.batch, 11)
    S = STORE[a.st]
    if a.st == "fp16":   # the module's own (float16) parameters
        p = {k: v.half().float() for k, v in p.items()}
    Y, attr, blocks = G.forward_taps(xt.to(dev).to(S), z.to(dev).to(S))
    torch.cuda.synchronize()
    rows = [0, 21, 42, 63][: max(1, min(4, a.batch))]
    ri = torch.tensor(rows)
    zr = z[ri].to(S).float()
    k = a.block
    prev = blocks[k - 2][ri].float().cpu()
    za = attr[k - 1][ri].float().cpu()
    g = blocks[k - 1][ri].float().cpu()
    with R.storage(S):
        e32 = R.gen_block_bf16_storage(prev, za, zr, p, "unet", 2, k)
    e64 = block64(prev, za, zr, p, k, a.st)
    e64f = block64(prev, za, zr, p, k, a.st, folded=True)
    print(f"AADBlk{k} {a.st} B={a.batch} rows={rows}: max|ref| {float(e32.abs().max()):.4f}")
    report("gpu vs emulation fp32", g, e32, a.st)
    report("gpu vs emulation fp64", g, e64, a.st)
    report("gpu vs fp64 folded mask", g, e64f, a.st)
    report("emu fp32 vs emu fp64", e32, e64, a.st)
    report("fp64 folded vs fp64", e64f, e64, a.st)


if __name__ == "__main__":
    main()

"""Weight packing: reference state_dict tensors -> the layouts the gfx950 kernels read.

Host-side tensor plumbing only (torch ops on the device, once per weight load).
Slot names are the ones ``ghost_aei_bind`` accepts (see aei_runtime.hip
``declare_slots``); INTEGRATION.md documents every layout.

Layouts (Npad = Cout rounded up to 128, Kpad = K rounded up to 32, zero padded):
  conv  [Cout,Cin,kh,kw]      -> [Npad][Kpad], K = (cb*kh*kw + ky*kw + kx)*32 + c%32 (cb = c/32) when
                                 Cin % 32 == 0, else (ky*kw + kx)*Cin + c
  conv3x3 to <= 3 channels    -> also [32][Kpad], row = (ky*3 + kx)*Cout + o, K = c  (narrow kernel)
  convT [Cin,Cout,4,4] (s2p1) -> [4][Npad][Kpad], phase = 2*py+px, K = (cb*4 + ty*2+tx)*32 + c%32,
                                 kernel tap ky = ((1,3),(0,2))[py][ty]  (sub-pixel decomposition)
  AAD conv1/conv2 (1x1)       -> [Npad][Kpad] rows interleaved per 16 channels: gamma c0..15,
                                 beta c0..15, gamma c16..31, ...  (+ the same for the biases)
                                 and, 16-bit (bf16 / fp16) with C in {64,128}: [C/64*128][Ca] rows permuted for the
                                 register-epilogue kernel (pack_aad_v3)
  all fc1/fc2 (Linear)        -> one fp32 [Npad][Kpad] = [gamma_l | beta_l] per AADLayer l in plan order
  up1 ConvT k2 on 1x1         -> fp32 [4096][Kpad], n = (y*2+x)*1024 + co
  BatchNorm (eval)            -> fp32 scale = g/sqrt(rv+eps), shift = b - rm*scale
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch

BN_EPS = 1e-5
_KTAP = ((1, 3), (0, 2))  # convT 4x4/s2/p1: kernel index of sub-pixel tap t at output parity p

ENC_DOWN = [(3, 32), (32, 64), (64, 128), (128, 256), (256, 512), (512, 1024), (1024, 1024)]
ENC_UP = {"unet": [(1024, 1024), (2048, 512), (1024, 256), (512, 128), (256, 64), (128, 32)],
          "linknet": [(1024, 1024), (1024, 512), (512, 256), (256, 128), (128, 64), (64, 32)]}
GEN_BLOCKS = {
    "unet": [(1024, 1024, 1024), (1024, 1024, 2048), (1024, 1024, 1024), (1024, 512, 512),
             (512, 256, 256), (256, 128, 128), (128, 64, 64), (64, 3, 64)],
    "linknet": [(1024, 1024, 1024), (1024, 1024, 1024), (1024, 1024, 512), (1024, 512, 256),
                (512, 256, 128), (256, 128, 64), (128, 64, 32), (64, 3, 32)],
}


GEN_BLOCKS["resnet"] = GEN_BLOCKS["unet"]   # AEI_Net.py:111-118: only linknet changes the generator


def rup(v: int, m: int) -> int:
    return (v + m - 1) // m * m


def pack_conv(w: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """K order (channel block of 32, tap, channel) when Cin % 32 == 0 — consecutive K steps are
    the taps of one channel block (input-row reuse in L1/L2); (tap, channel) otherwise."""
    co, ci, kh, kw = w.shape
    k = kh * kw * ci
    out = torch.zeros(rup(co, 128), rup(k, 32), dtype=dtype, device=w.device)
    if ci % 32 == 0:
        wk = w.reshape(co, ci // 32, 32, kh * kw).permute(0, 1, 3, 2)      # [co][cb][tap][c]
    else:
        wk = w.permute(0, 2, 3, 1)                                          # [co][ky][kx][c]
    out[:co, :k] = wk.reshape(co, k).to(dtype)
    return out


def pack_conv3x3_narrow(w: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """[Cout<=3, Cin, 3, 3] -> [32][Kpad]: row n = (ky*3 + kx)*Cout + o, K = input channel."""
    co, ci = w.shape[:2]
    assert co <= 3 and w.shape[2:] == (3, 3)
    out = torch.zeros(32, rup(ci, 32), dtype=dtype, device=w.device)
    out[:9 * co, :ci] = w.permute(2, 3, 0, 1).reshape(9 * co, ci).to(dtype)
    return out


def pack_convT4x4(w: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    ci, co = w.shape[:2]
    out = torch.zeros(4, rup(co, 128), rup(4 * ci, 32), dtype=dtype, device=w.device)
    for py in range(2):
        for px in range(2):
            taps = [w[:, :, _KTAP[py][ty], _KTAP[px][tx]].t() for ty in range(2) for tx in range(2)]
            blk = torch.stack(taps, 1)                                      # [co][tap][ci]
            if ci % 32 == 0:
                blk = blk.reshape(co, 4, ci // 32, 32).permute(0, 2, 1, 3)  # [co][cb][tap][c]
            out[2 * py + px, :co, :4 * ci] = blk.reshape(co, 4 * ci).to(dtype)
    return out


def bn_fold(sd: Dict[str, torch.Tensor], prefix: str, npad: int) -> Tuple[torch.Tensor, torch.Tensor]:
    g = sd[f"{prefix}.weight"].float()
    b = sd[f"{prefix}.bias"].float()
    rm = sd[f"{prefix}.running_mean"].float()
    rv = sd[f"{prefix}.running_var"].float()
    scale = g / torch.sqrt(rv + BN_EPS)
    shift = b - rm * scale
    s = torch.zeros(npad, dtype=torch.float32, device=g.device)
    t = torch.zeros(npad, dtype=torch.float32, device=g.device)
    s[:scale.numel()] = scale
    t[:shift.numel()] = shift
    return s, t


def interleave16(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """rows [a0..15, b0..15, a16..31, b16..31, ...] (the AAD GEMM's gamma/beta column pairs)."""
    c = a.shape[0]
    assert c % 16 == 0
    rest = a.shape[1:]
    return torch.stack([a.reshape(c // 16, 16, *rest), b.reshape(c // 16, 16, *rest)], 1).reshape(2 * c, *rest)


def pack_aad(sd, prefix: str, dtype) -> Dict[str, torch.Tensor]:
    w1 = sd[f"{prefix}.conv1.weight"]
    c, ca = w1.shape[:2]
    gb = interleave16(w1.reshape(c, ca), sd[f"{prefix}.conv2.weight"].reshape(c, ca))
    gbw = torch.zeros(rup(2 * c, 128), rup(ca, 32), dtype=dtype, device=w1.device)
    gbw[:2 * c, :ca] = gb.to(dtype)
    gbb = torch.zeros(rup(2 * c, 128), dtype=torch.float32, device=w1.device)
    gbb[:2 * c] = interleave16(sd[f"{prefix}.conv1.bias"].float(), sd[f"{prefix}.conv2.bias"].float())
    return {"gbw": gbw, "gbb": gbb,
            "wh": sd[f"{prefix}.conv_h.weight"].reshape(c).float().contiguous(),
            "bh": sd[f"{prefix}.conv_h.bias"].reshape(1).float().contiguous()}


def pack_aad_v3(sd, prefix: str, dtype) -> Dict[str, torch.Tensor]:
    """Weights of the register-epilogue AAD kernel (aad_v3.hip), C in {64, 128}.

    Per 64-channel tile, row rho = 16*i + 4*q + r (i = MFMA row tile, q = lane group, r = register)
    holds gamma (i < 4) or beta (i >= 4) of channel 32*((i>>1)&1) + 8*q + 4*(i&1) + r, so that a
    lane's accumulators are gamma/beta of 16 channels (two runs of 8) of one pixel.
    """
    w1 = sd[f"{prefix}.conv1.weight"]
    c, ca = w1.shape[:2]
    dev = w1.device
    rho = torch.arange(128, device=dev)
    i, q, r = rho >> 4, (rho >> 2) & 3, rho & 3
    gb = i >> 2
    cl = 32 * ((i >> 1) & 1) + 8 * q + 4 * (i & 1) + r
    W = [w1.reshape(c, ca), sd[f"{prefix}.conv2.weight"].reshape(c, ca)]
    Bs = [sd[f"{prefix}.conv1.bias"].float(), sd[f"{prefix}.conv2.bias"].float()]
    w3, b3 = [], []
    for ct in range(c // 64):
        ch = ct * 64 + cl
        w3.append(torch.where((gb == 0)[:, None], W[0][ch], W[1][ch]))
        b3.append(torch.where(gb == 0, Bs[0][ch], Bs[1][ch]))
    return {"w3": torch.cat(w3, 0).to(dtype).contiguous(), "b3": torch.cat(b3, 0).contiguous()}


def v3_layout(c: int, ca: int) -> bool:
    """AADLayers packed for the register-epilogue kernels too: aad_v3 (C in {64, 128}) and
    aad_wide (C in {256, 512, 1024}, Ca <= 512); mirrors aei_runtime.hip declare_slots."""
    return c in (64, 128) or (c in (256, 512, 1024) and ca <= 512)


def aad_plan(backbone: str, num_blocks: int) -> List[Tuple[str, str]]:
    """(slot prefix, state_dict prefix) of every AADLayer in the runtime's plan order."""
    out = []
    for k, (cin, cout, _) in enumerate(GEN_BLOCKS[backbone], 1):
        for i in range(num_blocks):
            out.append((f"gen.blk{k}.aad{i}", f"generator.AADBlk{k}.add_blocks.{3 * i}"))
        if cin != cout:
            out.append((f"gen.blk{k}.aadlast", f"generator.AADBlk{k}.last_add_block.0"))
    return out


RESNET_PLANES = [32, 64, 128, 256, 512, 256]   # resnet.py:93-98 (Bottleneck expansion 4)


def pack_resnet_encoder(sd, dtype) -> Dict[str, torch.Tensor]:
    """MLAttrEncoderResnet (resnet.py:81-149): every conv + its eval BatchNorm as scale/shift."""
    slots: Dict[str, torch.Tensor] = {}

    def conv_bn(slot, wkey, bnkey):
        w = sd[wkey]
        slots[f"{slot}.w"] = pack_conv(w, dtype)
        slots[f"{slot}.scale"], slots[f"{slot}.shift"] = bn_fold(sd, bnkey, rup(w.shape[0], 128))

    conv_bn("enc.r.conv0", "encoder.conv0.weight", "encoder.bn0")
    conv_bn("enc.r.conv1", "encoder.conv1.weight", "encoder.bn1")
    for li in range(1, 7):
        for blk in range(2):
            pre, slot = f"encoder.layer{li}.{blk}", f"enc.r.l{li}.b{blk}"
            for j in (1, 2, 3):
                conv_bn(f"{slot}.c{j}", f"{pre}.conv{j}.weight", f"{pre}.bn{j}")
            if blk == 0:
                conv_bn(f"{slot}.down", f"{pre}.downsample.0.weight", f"{pre}.downsample.1")
    return slots


def pack_all(sd: Dict[str, torch.Tensor], backbone: str, num_blocks: int, c_id: int,
             dtype: torch.dtype) -> Dict[str, torch.Tensor]:
    """Every runtime slot -> a contiguous device tensor."""
    if backbone not in GEN_BLOCKS:
        raise NotImplementedError(f"ghost_amd: backbone {backbone!r} has no MI355X path yet")
    slots: Dict[str, torch.Tensor] = {}
    if backbone == "resnet":
        slots.update(pack_resnet_encoder(sd, dtype))
    for i, (_ci, co) in enumerate(ENC_DOWN if backbone != "resnet" else [], 1):
        slots[f"enc.conv{i}.w"] = pack_conv(sd[f"encoder.conv{i}.0.weight"], dtype)
        s, t = bn_fold(sd, f"encoder.conv{i}.1", rup(co, 128))
        slots[f"enc.conv{i}.scale"], slots[f"enc.conv{i}.shift"] = s, t
    for i, (_ci, co) in enumerate(ENC_UP.get(backbone, []), 1):
        slots[f"enc.deconv{i}.w"] = pack_convT4x4(sd[f"encoder.deconv{i}.deconv.weight"], dtype)
        s, t = bn_fold(sd, f"encoder.deconv{i}.bn", rup(co, 128))
        slots[f"enc.deconv{i}.scale"], slots[f"enc.deconv{i}.shift"] = s, t
    # up1: ConvTranspose2d(c_id, 1024, k=2) on a 1x1 input
    w = sd["generator.up1.weight"].float()
    dev = w.device
    up = torch.zeros(4096, rup(c_id, 32), dtype=torch.float32, device=dev)
    up[:, :c_id] = w.permute(2, 3, 1, 0).reshape(4096, c_id)
    slots["gen.up1.w"] = up
    slots["gen.up1.shift"] = sd["generator.up1.bias"].float().repeat(4).contiguous()
    # AAD layers + the identity table
    ids_w, ids_b = [], []
    for slot, pre in aad_plan(backbone, num_blocks):
        for k, v in pack_aad(sd, pre, dtype).items():
            slots[f"{slot}.{k}"] = v
        if dtype in (torch.bfloat16, torch.float16) and v3_layout(*sd[f"{pre}.conv1.weight"].shape[:2]):
            for k, v in pack_aad_v3(sd, pre, dtype).items():
                slots[f"{slot}.{k}"] = v
        ids_w += [sd[f"{pre}.fc1.weight"].float(), sd[f"{pre}.fc2.weight"].float()]
        ids_b += [sd[f"{pre}.fc1.bias"].float(), sd[f"{pre}.fc2.bias"].float()]
    wid = torch.cat(ids_w, 0)
    ntot = wid.shape[0]
    idw = torch.zeros(rup(ntot, 128), rup(c_id, 32), dtype=torch.float32, device=dev)
    idw[:ntot, :c_id] = wid
    idb = torch.zeros(rup(ntot, 128), dtype=torch.float32, device=dev)
    idb[:ntot] = torch.cat(ids_b, 0)
    slots["gen.id.w"], slots["gen.id.shift"] = idw, idb
    # AAD_ResBlk 3x3 convs; the last one of a cin != cout block is fused with last_add_block's
    for k, (cin, cout, _) in enumerate(GEN_BLOCKS[backbone], 1):
        for i in range(num_blocks):
            w = sd[f"generator.AADBlk{k}.add_blocks.{3 * i + 2}.weight"]
            if i == num_blocks - 1 and cin != cout:
                w = torch.cat([w, sd[f"generator.AADBlk{k}.last_add_block.2.weight"]], 1)
            slots[f"gen.blk{k}.conv{i}.w"] = pack_conv(w, dtype)
            if w.shape[0] <= 3:
                slots[f"gen.blk{k}.conv{i}.wn"] = pack_conv3x3_narrow(w, dtype)
    return {k: v.contiguous() for k, v in slots.items()}

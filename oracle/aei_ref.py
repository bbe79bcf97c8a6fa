"""ORACLE — CPU restatement of GHOST's AEI_Net forward (test infrastructure only).

This module is the *checker* for the MI355X product path in ``ghost_amd``.  It is
imported only by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg; the product never imports, links or calls it, and there is
no CPU fallback in the product that routes through here.

It is a from-scratch restatement, written with ``torch.nn.functional`` ops on CPU
(fp32 by default, fp64 on request), of the reference algorithm:

* ``conv4x4``            -> /root/reference/network/AEI_Net.py:19-24
* ``deconv4x4``          -> /root/reference/network/AEI_Net.py:27-41
* ``MLAttrEncoder``      -> /root/reference/network/AEI_Net.py:44-95
* ``MLAttrEncoderResnet`` (backbone='resnet') -> /root/reference/network/resnet.py:43-149
* ``AADGenerator``       -> /root/reference/network/AEI_Net.py:98-139
* ``AEI_Net``            -> /root/reference/network/AEI_Net.py:143-159
* ``AADLayer.forward``   -> /root/reference/network/AADLayer.py:20-38
* ``AddBlocksSequential``-> /root/reference/network/AADLayer.py:40-50
* ``AAD_ResBlk``         -> /root/reference/network/AADLayer.py:53-80
* ``faceshifter_batch`` post-processing -> /root/reference/utils/inference/faceshifter_run.py:19-22
* ``transform_target_to_torch``        -> /root/reference/utils/inference/core.py:13-26

Parity status: PINNED.  ``tests/test_oracle_golden.py`` checks this restatement
against golden vectors produced by running the reference ``network.AEI_Net``
itself (``tests/golden/make_golden.py``, committed with its outputs).

Parameters are a flat ``{state_dict key: tensor}`` mapping with exactly the
reference's key names and torch layouts (Conv2d [Cout,Cin,kh,kw], ConvTranspose2d
[Cin,Cout,kh,kw], Linear [out,in]).
"""
from __future__ import annotations

import zlib
from typing import Dict, List, Tuple

import numpy as np
import torch
import torch.nn.functional as F

BN_EPS = 1e-5          # nn.BatchNorm2d default (AEI_Net.py:22,31)
IN_EPS = 1e-5          # nn.InstanceNorm2d default (AADLayer.py:16)
LRELU = 0.1            # AEI_Net.py:23,32

# ----------------------------------------------------------------------------
# architecture tables (AEI_Net.py:48-69, :101-118)
# ----------------------------------------------------------------------------
ENC_DOWN = [(3, 32), (32, 64), (64, 128), (128, 256), (256, 512), (512, 1024), (1024, 1024)]
ENC_UP = {
    "unet": [(1024, 1024), (2048, 512), (1024, 256), (512, 128), (256, 64), (128, 32)],
    "linknet": [(1024, 1024), (1024, 512), (512, 256), (256, 128), (128, 64), (64, 32)],
}
# (cin, cout, c_attr) per AADBlk1..8
GEN_BLOCKS = {
    "unet": [(1024, 1024, 1024), (1024, 1024, 2048), (1024, 1024, 1024), (1024, 512, 512),
             (512, 256, 256), (256, 128, 128), (128, 64, 64), (64, 3, 64)],
    # AEI_Net.py:111-118: every backbone but linknet takes the unet channel plan
    "resnet": [(1024, 1024, 1024), (1024, 1024, 2048), (1024, 1024, 1024), (1024, 512, 512),
               (512, 256, 256), (256, 128, 128), (128, 64, 64), (64, 3, 64)],
    "linknet": [(1024, 1024, 1024), (1024, 1024, 1024), (1024, 1024, 512), (1024, 512, 256),
                (512, 256, 128), (256, 128, 64), (128, 64, 32), (64, 3, 32)],
}


RESNET_PLANES = [32, 64, 128, 256, 512, 256]   # resnet.py:93-98, Bottleneck expansion 4


def resnet_blocks():
    """(layer, inplanes, planes, stride, block index) of MLAttrEncoderResnet (resnet.py:101-116, 147-149):
    two Bottlenecks per layer; the first has stride 2 (on its 1x1 conv1) and a 1x1/s2 + BN downsample."""
    out, inplanes = [], 64
    for li, planes in enumerate(RESNET_PLANES, 1):
        for blk in range(2):
            out.append((li, inplanes, planes, 2 if blk == 0 else 1, blk))
            inplanes = 4 * planes
    return out


def param_specs(backbone: str = "unet", num_blocks: int = 2, c_id: int = 512) -> List[Tuple[str, Tuple[int, ...], str]]:
    """Ordered (key, shape, kind) list matching the reference ``state_dict``.

    kind in {conv, convT, bn_w, bn_b, bn_rm, bn_rv, bn_nbt, lin_w, bias}.
    """
    if backbone not in GEN_BLOCKS:
        raise ValueError(f"backbone {backbone!r} not supported by the oracle")
    specs: List[Tuple[str, Tuple[int, ...], str]] = []

    def bn(prefix: str, c: int) -> None:
        specs.extend([(f"{prefix}.weight", (c,), "bn_w"), (f"{prefix}.bias", (c,), "bn_b"),
                      (f"{prefix}.running_mean", (c,), "bn_rm"), (f"{prefix}.running_var", (c,), "bn_rv"),
                      (f"{prefix}.num_batches_tracked", (), "bn_nbt")])

    if backbone == "resnet":
        # ResNet(Bottleneck, [2]*6) (resnet.py:81-149): stem conv0 7x7/s1, conv1 7x7/s2, six layers
        specs.append(("encoder.conv0.weight", (64, 3, 7, 7), "conv"))
        bn("encoder.bn0", 64)
        specs.append(("encoder.conv1.weight", (64, 64, 7, 7), "conv"))
        bn("encoder.bn1", 64)
        for li, cin, planes, stride, blk in resnet_blocks():
            pre = f"encoder.layer{li}.{blk}"
            specs.append((f"{pre}.conv1.weight", (planes, cin, 1, 1), "conv"))
            bn(f"{pre}.bn1", planes)
            specs.append((f"{pre}.conv2.weight", (planes, planes, 3, 3), "conv"))
            bn(f"{pre}.bn2", planes)
            specs.append((f"{pre}.conv3.weight", (4 * planes, planes, 1, 1), "conv"))
            bn(f"{pre}.bn3", 4 * planes)
            if blk == 0:
                specs.append((f"{pre}.downsample.0.weight", (4 * planes, cin, 1, 1), "conv"))
                bn(f"{pre}.downsample.1", 4 * planes)
    else:
        for i, (ci, co) in enumerate(ENC_DOWN, 1):
            specs.append((f"encoder.conv{i}.0.weight", (co, ci, 4, 4), "conv"))
            bn(f"encoder.conv{i}.1", co)
        for i, (ci, co) in enumerate(ENC_UP[backbone], 1):
            specs.append((f"encoder.deconv{i}.deconv.weight", (ci, co, 4, 4), "convT"))
            bn(f"encoder.deconv{i}.bn", co)
    specs.append(("generator.up1.weight", (c_id, 1024, 2, 2), "convT"))
    specs.append(("generator.up1.bias", (1024,), "bias"))

    def aad(prefix: str, c_x: int, c_attr: int) -> None:
        specs.extend([(f"{prefix}.conv1.weight", (c_x, c_attr, 1, 1), "conv"), (f"{prefix}.conv1.bias", (c_x,), "bias"),
                      (f"{prefix}.conv2.weight", (c_x, c_attr, 1, 1), "conv"), (f"{prefix}.conv2.bias", (c_x,), "bias"),
                      (f"{prefix}.fc1.weight", (c_x, c_id), "lin_w"), (f"{prefix}.fc1.bias", (c_x,), "bias"),
                      (f"{prefix}.fc2.weight", (c_x, c_id), "lin_w"), (f"{prefix}.fc2.bias", (c_x,), "bias"),
                      (f"{prefix}.conv_h.weight", (1, c_x, 1, 1), "conv"), (f"{prefix}.conv_h.bias", (1,), "bias")])

    for k, (cin, cout, ca) in enumerate(GEN_BLOCKS[backbone], 1):
        p = f"generator.AADBlk{k}"
        for i in range(num_blocks):
            out = cin if i < num_blocks - 1 else cout
            aad(f"{p}.add_blocks.{3 * i}", cin, ca)
            specs.append((f"{p}.add_blocks.{3 * i + 2}.weight", (out, cin, 3, 3), "conv"))
        if cin != cout:
            aad(f"{p}.last_add_block.0", cin, ca)
            specs.append((f"{p}.last_add_block.2.weight", (cout, cin, 3, 3), "conv"))
    return specs


def make_weights(specs, dtype=torch.float32) -> Dict[str, torch.Tensor]:
    """Deterministic key-hashed weight recipe.

    Every float key seeds ``np.random.Generator(PCG64(crc32(key)))``:
    conv/convT ~ N(0, sqrt(2/(fan_in+fan_out))); linear weights and biases ~ N(0, 0.02);
    BN gamma ~ U(0.5,1.5), beta ~ N(0,0.1), running_mean ~ N(0,0.1), running_var ~ U(0.5,1.5).
    """
    out: Dict[str, torch.Tensor] = {}
    for key, shape, kind in specs:
        if kind == "bn_nbt":
            out[key] = torch.zeros((), dtype=torch.int64)
            continue
        g = np.random.Generator(np.random.PCG64(zlib.crc32(key.encode())))
        if kind in ("conv", "convT"):
            rf = int(np.prod(shape[2:]))
            std = float(np.sqrt(2.0 / ((shape[0] + shape[1]) * rf)))
            a = g.normal(0.0, std, size=shape)
        elif kind in ("lin_w", "bias"):
            a = g.normal(0.0, 0.02, size=shape)
        elif kind == "bn_w" or kind == "bn_rv":
            a = g.uniform(0.5, 1.5, size=shape)
        elif kind in ("bn_b", "bn_rm"):
            a = g.normal(0.0, 0.1, size=shape)
        else:  # pragma: no cover
            raise ValueError(kind)
        out[key] = torch.from_numpy(np.asarray(a, dtype=np.float32)).to(dtype)
    return out


def make_inputs(batch: int, seed: int = 7, c_id: int = 512):
    """Xt ~ U(-1,1) [B,3,256,256], z_id ~ N(0,1) [B,c_id] from PCG64(seed)."""
    g = np.random.Generator(np.random.PCG64(seed))
    xt = g.uniform(-1.0, 1.0, size=(batch, 3, 256, 256)).astype(np.float32)
    z = g.normal(0.0, 1.0, size=(batch, c_id)).astype(np.float32)
    return torch.from_numpy(xt), torch.from_numpy(z)


def make_u8_crops(batch: int, seed: int = 0) -> np.ndarray:
    """Synthetic aligned-face crops: uint8 BGR NHWC [B,256,256,3] ~ U{0..255}."""
    g = np.random.Generator(np.random.PCG64(seed))
    return g.integers(0, 256, size=(batch, 256, 256, 3), dtype=np.uint8)


# ----------------------------------------------------------------------------
# ops
# ----------------------------------------------------------------------------
def _bn_eval(x, p, prefix):
    # eval-mode BatchNorm with running statistics (AEI_Net.py:22,31)
    return F.batch_norm(x, p[f"{prefix}.running_mean"].to(x.dtype), p[f"{prefix}.running_var"].to(x.dtype),
                        p[f"{prefix}.weight"].to(x.dtype), p[f"{prefix}.bias"].to(x.dtype), False, 0.0, BN_EPS)


def conv4x4_block(x, p, i):
    """Conv4x4/s2/p1 (no bias) -> BN(eval) -> LeakyReLU(0.1)   (AEI_Net.py:19-24)."""
    y = F.conv2d(x, p[f"encoder.conv{i}.0.weight"].to(x.dtype), None, stride=2, padding=1)
    return F.leaky_relu(_bn_eval(y, p, f"encoder.conv{i}.1"), LRELU)


def deconv4x4_block(x, skip, p, i, backbone):
    """ConvT4x4/s2/p1 -> BN -> LReLU -> cat((x,skip),1) | x+skip   (AEI_Net.py:27-41)."""
    y = F.conv_transpose2d(x, p[f"encoder.deconv{i}.deconv.weight"].to(x.dtype), None, stride=2, padding=1)
    y = F.leaky_relu(_bn_eval(y, p, f"encoder.deconv{i}.bn"), LRELU)
    return y + skip if backbone == "linknet" else torch.cat((y, skip), dim=1)


def up2x(x):
    """Bilinear x2, align_corners=True (AEI_Net.py:94,125-137)."""
    return F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=True)


def _bottleneck(x, p, pre, stride, has_down):
    """Bottleneck.forward (resnet.py:57-78): 1x1/s -> BN -> ReLU -> 3x3 -> BN -> ReLU -> 1x1 -> BN, + residual, ReLU."""
    out = F.relu(_bn_eval(F.conv2d(x, p[f"{pre}.conv1.weight"].to(x.dtype), None, stride=stride), p, f"{pre}.bn1"))
    out = F.relu(_bn_eval(F.conv2d(out, p[f"{pre}.conv2.weight"].to(x.dtype), None, padding=1), p, f"{pre}.bn2"))
    out = _bn_eval(F.conv2d(out, p[f"{pre}.conv3.weight"].to(x.dtype), None), p, f"{pre}.bn3")
    res = x
    if has_down:
        res = _bn_eval(F.conv2d(x, p[f"{pre}.downsample.0.weight"].to(x.dtype), None, stride=stride), p,
                       f"{pre}.downsample.1")
    return F.relu(out + res)


def encoder_resnet(xt, p):
    """ResNet.forward (resnet.py:122-144) -> (x7, x6, x5, x4, x3, x2, x1, x0)."""
    x0 = F.relu(_bn_eval(F.conv2d(xt, p["encoder.conv0.weight"].to(xt.dtype), None, padding=3), p, "encoder.bn0"))
    x = F.relu(_bn_eval(F.conv2d(x0, p["encoder.conv1.weight"].to(xt.dtype), None, stride=2, padding=3), p,
                        "encoder.bn1"))
    feats = [x0, x]
    for li, _cin, _planes, stride, blk in resnet_blocks():
        x = _bottleneck(x, p, f"encoder.layer{li}.{blk}", stride, blk == 0)
        if blk == 1:
            feats.append(x)
    return tuple(reversed(feats))


def encoder(xt, p, backbone="unet"):
    """MLAttrEncoder.forward (AEI_Net.py:72-95) -> 8-tuple z_attr1..z_attr8."""
    if backbone == "resnet":
        return encoder_resnet(xt, p)
    feats = []
    x = xt
    for i in range(1, 8):
        x = conv4x4_block(x, p, i)
        feats.append(x)
    z = [feats[6]]
    for i in range(1, 7):
        z.append(deconv4x4_block(z[-1], feats[6 - i], p, i, backbone))
    z.append(up2x(z[-1]))
    return tuple(z)


def aad_layer(h_in, z_attr, z_id, p, prefix):
    """AADLayer.forward (AADLayer.py:20-38): IN, gamma/beta from attr (1x1) and id (Linear), sigmoid mask blend."""
    dt = h_in.dtype
    h = F.instance_norm(h_in, eps=IN_EPS)
    ga = F.conv2d(z_attr, p[f"{prefix}.conv1.weight"].to(dt), p[f"{prefix}.conv1.bias"].to(dt))
    ba = F.conv2d(z_attr, p[f"{prefix}.conv2.weight"].to(dt), p[f"{prefix}.conv2.bias"].to(dt))
    gi = F.linear(z_id, p[f"{prefix}.fc1.weight"].to(dt), p[f"{prefix}.fc1.bias"].to(dt))
    bi = F.linear(z_id, p[f"{prefix}.fc2.weight"].to(dt), p[f"{prefix}.fc2.bias"].to(dt))
    c_x = h.shape[1]
    A = ga * h + ba
    I = gi.reshape(h.shape[0], c_x, 1, 1) * h + bi.reshape(h.shape[0], c_x, 1, 1)
    M = torch.sigmoid(F.conv2d(h, p[f"{prefix}.conv_h.weight"].to(dt), p[f"{prefix}.conv_h.bias"].to(dt)))
    return (1 - M) * A + M * I


def _add_seq(h, z_attr, z_id, p, prefix, n_layers):
    # AddBlocksSequential (AADLayer.py:40-50): every AADLayer sees the same z_attr / z_id
    x = h
    for i in range(n_layers):
        x = aad_layer(x, z_attr, z_id, p, f"{prefix}.{3 * i}")
        x = F.relu(x)
        x = F.conv2d(x, p[f"{prefix}.{3 * i + 2}.weight"].to(x.dtype), None, padding=1)
    return x


def aad_resblk(h, z_attr, z_id, p, k, cin, cout, num_blocks):
    """AAD_ResBlk.forward (AADLayer.py:74-80): x = add_blocks(h); h' = last_add_block(h) if cin != cout; x + h'."""
    prefix = f"generator.AADBlk{k}"
    x = _add_seq(h, z_attr, z_id, p, f"{prefix}.add_blocks", num_blocks)
    if cin != cout:
        h = _add_seq(h, z_attr, z_id, p, f"{prefix}.last_add_block", 1)
    return x + h


def generator(z_attr, z_id, p, backbone="unet", num_blocks=2):
    """AADGenerator.forward (AEI_Net.py:122-139)."""
    dt = z_attr[0].dtype
    z_id = z_id.to(dt).reshape(z_id.shape[0], -1)
    m = F.conv_transpose2d(z_id.reshape(z_id.shape[0], -1, 1, 1), p["generator.up1.weight"].to(dt),
                           p["generator.up1.bias"].to(dt))
    for k, (cin, cout, _ca) in enumerate(GEN_BLOCKS[backbone], 1):
        y = aad_resblk(m, z_attr[k - 1], z_id, p, k, cin, cout, num_blocks)
        m = up2x(y) if k < 8 else y
    return torch.tanh(m)


@torch.no_grad()
def aei_forward(p, xt, z_id, backbone="unet", num_blocks=2, dtype=torch.float32):
    """AEI_Net.forward (AEI_Net.py:153-156) -> (Y, attr)."""
    xt = xt.to(dtype)
    attr = encoder(xt, p, backbone)
    return generator(attr, z_id, p, backbone, num_blocks), attr


# ----------------------------------------------------------------------------
# bf16-storage emulation (the checker of the bf16 throughput path)
# ----------------------------------------------------------------------------
# The same reference algorithm as above, with every tensor the MI355X runtime *stores* in bf16
# rounded to bf16 at that point, and every weight the packer stores in bf16 rounded likewise
# (ghost_amd/network/pack.py).  Arithmetic between storage points stays fp32: the kernels
# accumulate in fp32 and apply BatchNorm / bias / InstanceNorm / mask / blend / residual / tanh
# in fp32 epilogues.  Differences left against the kernels are fp32 summation order only, which
# can flip a bf16 rounding here and there; the GPU tests gate on that residual.
#
# Storage points (aei_runtime.hip plan):
#   input x (crops_kernel / input_to_nhwc)            -> bf16
#   every encoder conv / deconv output after BN + LReLU (+ linknet skip add) -> bf16
#   z_attr8 = up2x(z_attr7)                           -> bf16
#   m1 = up1(z_id) (fp32 weights, fp32 z_id)         -> bf16
#   AADLayer output after its ReLU                    -> bf16   (gamma/beta from bf16 conv1/conv2,
#                                                                fc1/fc2 and conv_h in fp32)
#   3x3 conv outputs inside a block                   -> bf16
#   block output: last conv + residual (x + h' in one GEMM over [a_x | a_h] when cin != cout) -> bf16
#   m_{k+1} = up2x(y_k)                               -> bf16 (materialised or sampled in-kernel)
#   Y = tanh(.)                                       -> bf16; the u8 frame comes from the fp32 tanh
# InstanceNorm statistics are those of the stored bf16 tensor, except where the runtime takes the
# statistics of an upsample in closed form over its source (source side >= 32, C % 64 == 0:
# ops.hip in_stats_up2x_closed_form), which are the statistics of the fp32 upsample.
_STORE = [torch.bfloat16]     # storage dtype of the emulation (float32: rounding off, for self-checks)
# GHOST_AEI_OPT_TAP_PARTIALS of the runtime being emulated (include/ghost_amd.h): AADBlk8's 3x3 conv to 3
# channels contracted per tap in its producers, each tap's partial sum stored in fp16 (2: the h path and
# last_add_block's x', 1: the h path only, 0: neither)
_TAP_PARTIALS = [2]


def _q(t: torch.Tensor) -> torch.Tensor:
    return t.to(_STORE[0]).float()


def _wq(p, key):
    return _q(p[key].float())


def _conv4x4_block_q(x, p, i):
    y = F.conv2d(x, _wq(p, f"encoder.conv{i}.0.weight"), None, stride=2, padding=1)
    return _q(F.leaky_relu(_bn_eval(y, p, f"encoder.conv{i}.1"), LRELU))


def _deconv4x4_block_q(x, skip, p, i, backbone):
    y = F.conv_transpose2d(x, _wq(p, f"encoder.deconv{i}.deconv.weight"), None, stride=2, padding=1)
    y = F.leaky_relu(_bn_eval(y, p, f"encoder.deconv{i}.bn"), LRELU)
    return _q(y + skip) if backbone == "linknet" else torch.cat((_q(y), skip), dim=1)


def _res_conv_q(x, p, wkey, bnkey, stride, pad, relu, res=None):
    y = _bn_eval(F.conv2d(x, _wq(p, wkey), None, stride=stride, padding=pad), p, bnkey)
    if res is not None:
        y = y + res
    return _q(F.relu(y) if relu else y)


def _encoder_resnet_q(xt, p):
    x0 = _res_conv_q(xt, p, "encoder.conv0.weight", "encoder.bn0", 1, 3, True)
    x = _res_conv_q(x0, p, "encoder.conv1.weight", "encoder.bn1", 2, 3, True)
    feats = [x0, x]
    for li, _cin, _planes, stride, blk in resnet_blocks():
        pre = f"encoder.layer{li}.{blk}"
        t = _res_conv_q(x, p, f"{pre}.conv1.weight", f"{pre}.bn1", stride, 0, True)
        t = _res_conv_q(t, p, f"{pre}.conv2.weight", f"{pre}.bn2", 1, 1, True)
        res = x
        if blk == 0:
            res = _res_conv_q(x, p, f"{pre}.downsample.0.weight", f"{pre}.downsample.1", stride, 0, False)
        x = _res_conv_q(t, p, f"{pre}.conv3.weight", f"{pre}.bn3", 1, 0, True, res)
        if blk == 1:
            feats.append(x)
    return tuple(reversed(feats))


def encoder_bf16_storage(xt, p, backbone="unet"):
    """MLAttrEncoder.forward (AEI_Net.py:72-95) with bf16 storage; xt already bf16-valued."""
    if backbone == "resnet":
        return _encoder_resnet_q(xt, p)
    feats, x = [], xt
    for i in range(1, 8):
        x = _conv4x4_block_q(x, p, i)
        feats.append(x)
    z = [feats[6]]
    for i in range(1, 7):
        z.append(_deconv4x4_block_q(z[-1], feats[6 - i], p, i, backbone))
    z.append(_q(up2x(z[-1])))
    return tuple(z)


def _in_stats(t):
    var, mean = torch.var_mean(t, dim=(2, 3), unbiased=False, keepdim=True)
    return mean, torch.rsqrt(var + IN_EPS)


def aad_layer_bf16_storage(h_in, z_attr, z_id, p, prefix, stats=None):
    """AADLayer.forward (AADLayer.py:20-38) + the ReLU after it, bf16 weights for conv1/conv2,
    output stored in bf16.  `stats` = (mean, rstd) when the runtime takes them elsewhere."""
    mean, rstd = stats if stats is not None else _in_stats(h_in)
    h = (h_in - mean) * rstd
    ga = F.conv2d(z_attr, _wq(p, f"{prefix}.conv1.weight"), p[f"{prefix}.conv1.bias"].float())
    ba = F.conv2d(z_attr, _wq(p, f"{prefix}.conv2.weight"), p[f"{prefix}.conv2.bias"].float())
    gi = F.linear(z_id, p[f"{prefix}.fc1.weight"].float(), p[f"{prefix}.fc1.bias"].float())
    bi = F.linear(z_id, p[f"{prefix}.fc2.weight"].float(), p[f"{prefix}.fc2.bias"].float())
    c_x = h.shape[1]
    A = ga * h + ba
    I = gi.reshape(h.shape[0], c_x, 1, 1) * h + bi.reshape(h.shape[0], c_x, 1, 1)
    M = torch.sigmoid(F.conv2d(h, p[f"{prefix}.conv_h.weight"].float(), p[f"{prefix}.conv_h.bias"].float()))
    return _q(F.relu((1 - M) * A + M * I))


def up1_bf16_storage(z_id, p):
    """m1 = up1(z_id) (AEI_Net.py:101,123): fp32 weights and z_id, stored in bf16."""
    z_id = z_id.float().reshape(z_id.shape[0], -1)
    return _q(F.conv_transpose2d(z_id.reshape(z_id.shape[0], -1, 1, 1), p["generator.up1.weight"].float(),
                                 p["generator.up1.bias"].float()))


def _tap_conv3x3(a, w, round16):
    """conv2d(a, w, padding=1) for 3 output channels as the runtime's tap-partial path computes it
    (ghost_amd/csrc/tap_rows.h): per tap (dy, dx) the partial sum Z = sum_c w[:, c, dy, dx] * a_c at every
    source pixel (fp32 over bf16 operands).  round16 False: out = sum over taps, unrounded (the narrow conv's
    own channels).  round16 True: the producer's fp16 row sums inside 8-column segments,
    R_dy(x) = (Z_{dy,0}(x-1) + Z_{dy,1}(x)) + Z_{dy,2}(x+1) (neighbours across a segment end left out), plus the
    fp16 segment-end terms at columns 8j - 1 (Z_{dy,2} of column 8j) and 8j (Z_{dy,0} of column 8j - 1);
    out(y, x) = sum_dy of those at source row y + dy - 1 (zero outside)."""
    H, W = a.shape[-2:]
    z = [[torch.einsum("bchw,oc->bohw", a, w[:, :, dy, dx]) for dx in range(3)] for dy in range(3)]
    out = torch.zeros(a.shape[0], w.shape[0], H, W)
    if not round16:
        for dy in range(3):
            for dx in range(3):
                out = out + F.pad(z[dy][dx], (1, 1, 1, 1))[:, :, dy:dy + H, dx:dx + W]
        return out
    col = torch.arange(W) % 8
    for dy in range(3):
        from_left = F.pad(z[dy][0], (1, 0))[..., :W]     # Z_{dy,0}(x - 1), zero at x = 0
        from_right = F.pad(z[dy][2], (0, 1))[..., 1:]    # Z_{dy,2}(x + 1), zero at x = W - 1
        zero = torch.zeros(())
        r = ((torch.where(col != 0, from_left, zero) + z[dy][1]) + torch.where(col != 7, from_right, zero))
        ends = torch.where(col == 7, from_right.half().float(), torch.where(col == 0, from_left.half().float(), zero))
        c = r.half().float() + ends
        out = out + F.pad(c, (0, 0, 1, 1))[:, :, dy:dy + H, :]
    return out


def gen_block_bf16_storage(y_prev, za, z_id, p, backbone, num_blocks, k):
    """AADBlk_k (AAD_ResBlk.forward, AADLayer.py:74-80) from the *stored* previous block output
    (k = 1: m1 from up1_bf16_storage), including the x2 upsample in front of it (AEI_Net.py:125-137).
    Returns the stored block output (bf16-valued; k = 8: the fp32 pre-tanh sum).  Taking the stored
    input of one block isolates that block's arithmetic: the per-stage parity tests feed it the
    GPU's own AADBlk_{k-1} output."""
    cin, cout, _ca = GEN_BLOCKS[backbone][k - 1]
    z_id = z_id.float().reshape(z_id.shape[0], -1)
    if k == 1:
        m, m_stats = y_prev, None
    else:
        u = up2x(y_prev)
        m = _q(u)
        m_stats = _in_stats(u) if (y_prev.shape[-1] >= 32 and cin % 64 == 0) else None
    pre = f"generator.AADBlk{k}"
    x, st = m, m_stats
    zp = _TAP_PARTIALS[0] if (k == 8 and cin != cout and cin == 64 and cout == 3
                              and _STORE[0] in (torch.bfloat16, torch.float16)) else 0
    for i in range(num_blocks):
        a = aad_layer_bf16_storage(x, za, z_id, p, f"{pre}.add_blocks.{3 * i}", st)
        wc = _wq(p, f"{pre}.add_blocks.{3 * i + 2}.weight")
        x = _tap_conv3x3(a, wc, True) if (zp and i == num_blocks - 1) else F.conv2d(a, wc, None, padding=1)
        st = None
        if i < num_blocks - 1:
            x = _q(x)
    if cin != cout:
        a = aad_layer_bf16_storage(m, za, z_id, p, f"{pre}.last_add_block.0", m_stats)
        wl = _wq(p, f"{pre}.last_add_block.2.weight")
        y = x + (_tap_conv3x3(a, wl, zp == 2) if zp else F.conv2d(a, wl, None, padding=1))
    else:
        y = x + m
    return y if k == 8 else _q(y)


def generator_bf16_storage(z_attr, z_id, p, backbone="unet", num_blocks=2):
    """AADGenerator.forward (AEI_Net.py:122-139) with bf16 storage -> (tanh fp32, [y_1 .. y_8] block
    outputs as stored, y_8 the pre-tanh sum)."""
    y = up1_bf16_storage(z_id, p)
    blocks = []
    for k in range(1, 9):
        y = gen_block_bf16_storage(y, z_attr[k - 1], z_id, p, backbone, num_blocks, k)
        blocks.append(y)
    return torch.tanh(blocks[-1]), blocks


@torch.no_grad()
def aei_forward_bf16_storage(p, xt, z_id, backbone="unet", num_blocks=2, store=torch.bfloat16, tap_partials=2):
    """AEI_Net.forward (AEI_Net.py:153-156) as the bf16 runtime stores it -> (Y, attr, blocks, y_u8_src).

    Y is the bf16-rounded tanh output, attr the stored encoder maps, blocks the stored AADBlk1..7
    outputs (+ AADBlk8's pre-tanh sum), and y_u8_src the fp32 tanh the uint8 frame is made from.
    tap_partials: the runtime's GHOST_AEI_OPT_TAP_PARTIALS (fp16 per-tap partials of AADBlk8's output conv)."""
    prev, _STORE[0] = _STORE[0], store
    prev_tp, _TAP_PARTIALS[0] = _TAP_PARTIALS[0], tap_partials
    try:
        xt = _q(xt.float())
        attr = encoder_bf16_storage(xt, p, backbone)
        t, blocks = generator_bf16_storage(attr, z_id, p, backbone, num_blocks)
        return _q(t), attr, blocks, t
    finally:
        _STORE[0] = prev
        _TAP_PARTIALS[0] = prev_tp


def aei_forward_fp16_storage(p, xt, z_id, backbone="unet", num_blocks=2, tap_partials=2):
    """The fp16-storage runtime (a .half() module, inference.py:30): the same emulation with every stored
    tensor rounded to float16 instead of bfloat16 (fp32 arithmetic in between, as the kernels)."""
    return aei_forward_bf16_storage(p, xt, z_id, backbone, num_blocks, store=torch.float16, tap_partials=tap_partials)


class storage:
    """``with aei_ref.storage(torch.float16, tap_partials=2):`` — the per-stage emulation functions
    (gen_block_bf16_storage, aad_layer_bf16_storage, up1_bf16_storage ...) round to this dtype inside."""

    def __init__(self, dtype, tap_partials=2):
        self.dtype, self.tp = dtype, tap_partials

    def __enter__(self):
        self.prev = (_STORE[0], _TAP_PARTIALS[0])
        _STORE[0], _TAP_PARTIALS[0] = self.dtype, self.tp
        return self

    def __exit__(self, *exc):
        _STORE[0], _TAP_PARTIALS[0] = self.prev
        return False


def fp16_reference_forward(p, xt, z_id, backbone="unet", num_blocks=2):
    """The reference GPU precision (inference.py:30 G.half(), core.py:21,66 fp16 inputs): the same
    restatement evaluated in float16 end to end (CPU fp16 ops), returned as fp32."""
    p16 = {k: (v.half() if v.is_floating_point() else v) for k, v in p.items()}
    y, _ = aei_forward(p16, xt.half(), z_id.half(), backbone, num_blocks, dtype=torch.float16)
    return y.float()


# ----------------------------------------------------------------------------
# pipeline arithmetic on either side of the generator
# ----------------------------------------------------------------------------
def transform_target(crops_u8_bgr: np.ndarray) -> torch.Tensor:
    """transform_target_to_torch(half=False) (core.py:13-26): BGR->RGB, /255, (x-0.5)/0.5, NHWC->NCHW view."""
    t = torch.from_numpy(crops_u8_bgr.copy())[:, :, :, [2, 1, 0]] / 255.0
    t = (t - 0.5) / 0.5
    return t.permute(0, 3, 1, 2)


def y_to_u8_bgr(y: torch.Tensor) -> np.ndarray:
    """faceshifter_batch post-processing (faceshifter_run.py:20-22): ((Y*0.5+0.5)*255)[..., BGR] -> uint8 (trunc)."""
    t = (y.permute(0, 2, 3, 1) * 0.5 + 0.5) * 255
    return t[:, :, :, [2, 1, 0]].type(torch.uint8).numpy()

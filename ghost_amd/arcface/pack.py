"""IResNet state_dict -> the slots of arc_runtime.hip (layouts as ghost_amd/network/pack.py)."""
from __future__ import annotations

from typing import Dict

import torch

from ..network.pack import bn_fold, pack_conv, rup

WIDTHS = (64, 128, 256, 512)


def pack_iresnet(sd: Dict[str, torch.Tensor], layers, dtype) -> Dict[str, torch.Tensor]:
    slots: Dict[str, torch.Tensor] = {}

    def bn(slot, key, n):
        slots[f"{slot}.scale"], slots[f"{slot}.shift"] = bn_fold(sd, key, rup(n, 128))

    def prelu(slot, key, n):
        t = torch.zeros(rup(n, 128), dtype=torch.float32, device=sd[key].device)
        t[:n] = sd[key].float().reshape(-1)
        slots[slot] = t

    slots["stem.w"] = pack_conv(sd["conv1.weight"], dtype)
    bn("stem.bn", "bn1", 64)
    prelu("stem.prelu", "prelu.weight", 64)
    inp = 64
    for li, (planes, n) in enumerate(zip(WIDTHS, layers), 1):
        for b in range(n):
            pre, nm = f"layer{li}.{b}", f"l{li}.b{b}"
            bn(f"{nm}.bn1", f"{pre}.bn1", inp)
            slots[f"{nm}.c1.w"] = pack_conv(sd[f"{pre}.conv1.weight"], dtype)
            bn(f"{nm}.bn2", f"{pre}.bn2", planes)
            prelu(f"{nm}.prelu", f"{pre}.prelu.weight", planes)
            slots[f"{nm}.c2.w"] = pack_conv(sd[f"{pre}.conv2.weight"], dtype)
            bn(f"{nm}.bn3", f"{pre}.bn3", planes)
            if b == 0:
                slots[f"{nm}.down.w"] = pack_conv(sd[f"{pre}.downsample.0.weight"], dtype)
                bn(f"{nm}.down", f"{pre}.downsample.1", planes)
            inp = planes
    bn("head.bn2", "bn2", 512)
    # fc over torch.flatten of NCHW [N,512,7,7] (feature index c*49 + y*7 + x) == a 7x7 valid conv
    fw = sd["fc.weight"]
    nf = fw.shape[0]
    slots["fc.w"] = pack_conv(fw.reshape(nf, 512, 7, 7), dtype)
    # features = BatchNorm1d(fc(x)): scale = g/sqrt(rv+eps), shift = (b_fc - rm)*scale + beta
    g, beta = sd["features.weight"].float(), sd["features.bias"].float()
    rm, rv = sd["features.running_mean"].float(), sd["features.running_var"].float()
    sc = g / torch.sqrt(rv + 1e-5)
    sh = (sd["fc.bias"].float() - rm) * sc + beta
    s = torch.zeros(rup(nf, 128), dtype=torch.float32, device=fw.device)
    t = torch.zeros(rup(nf, 128), dtype=torch.float32, device=fw.device)
    s[:nf], t[:nf] = sc, sh
    slots["fc.scale"], slots["fc.shift"] = s, t
    return {k: v.contiguous() for k, v in slots.items()}

"""Drop-in for network/AADLayer.py on MI355X.

Same classes, constructor arguments, submodule names and state_dict keys as the
reference (network/AADLayer.py:5-80), so reference checkpoints load unchanged.
The modules are parameter containers: execution goes through the native library.
``AADLayer.forward`` runs the fused gfx950 AAD kernels (IN statistics, sigmoid mask,
1x1 gamma/beta GEMM with the blend epilogue); the block containers are executed as a
whole by ``AEI_Net.forward`` (see AEI_Net.py) and refuse per-module torch execution.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import _lib
from .pack import pack_aad, rup


class AADLayer(nn.Module):
    """AADLayer(c_x, attr_c, c_id)  (AADLayer.py:5-18); forward = AADLayer.py:20-38."""

    def __init__(self, c_x, attr_c, c_id):
        super().__init__()
        self.attr_c = attr_c
        self.c_id = c_id
        self.c_x = c_x
        self.conv1 = nn.Conv2d(attr_c, c_x, kernel_size=1, stride=1, padding=0, bias=True)
        self.conv2 = nn.Conv2d(attr_c, c_x, kernel_size=1, stride=1, padding=0, bias=True)
        self.fc1 = nn.Linear(c_id, c_x)
        self.fc2 = nn.Linear(c_id, c_x)
        self.norm = nn.InstanceNorm2d(c_x, affine=False)
        self.conv_h = nn.Conv2d(c_x, 1, kernel_size=1, stride=1, padding=0, bias=True)
        self._pack_cache = None

    def _packed(self, dtype):
        sig = (dtype,) + tuple((p.data_ptr(), p._version) for p in self.parameters())
        if self._pack_cache is None or self._pack_cache[0] != sig:
            sd = {k: v.detach() for k, v in self.state_dict().items()}
            p = pack_aad({"l." + k: v for k, v in sd.items()}, "l", dtype)
            idw = torch.cat([self.fc1.weight, self.fc2.weight], 0).detach().float()
            idwp = torch.zeros(rup(2 * self.c_x, 128), rup(self.c_id, 32), dtype=torch.float32, device=idw.device)
            idwp[:2 * self.c_x, :self.c_id] = idw
            idb = torch.zeros(rup(2 * self.c_x, 128), dtype=torch.float32, device=idw.device)
            idb[:2 * self.c_x] = torch.cat([self.fc1.bias, self.fc2.bias]).detach().float()
            p["idw"], p["idb"] = idwp, idb
            self._pack_cache = (sig, p)
        return self._pack_cache[1]

    @torch.no_grad()
    def forward(self, h_in, z_attr, z_id, relu: bool = False):
        _lib.require_gpu(h_in, "AADLayer.forward")
        _lib.require_same_device(z_attr, h_in.device, "z_attr")
        _lib.require_same_device(z_id, h_in.device, "z_id")
        lib = _lib.load()
        pdt = self.conv1.weight.dtype
        dt = torch.float32 if pdt == torch.float32 else torch.bfloat16
        p = self._packed(dt)
        B, C, H, W = h_in.shape
        Ca = z_attr.shape[1]
        dev = h_in.device
        h = h_in.to(dt).contiguous(memory_format=torch.channels_last)        # NHWC storage
        za = z_attr.to(dt).contiguous(memory_format=torch.channels_last)
        zid = z_id.reshape(B, -1).float().contiguous()
        s = _lib.stream_ptr(dev)
        idgb = torch.empty(B, 2 * C, dtype=torch.float32, device=dev)
        ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
        _lib.check(lib.ghost_linear_f32(zid.data_ptr(), B, self.c_id, p["idw"].data_ptr(), 2 * C, p["idw"].shape[0],
                                        p["idw"].shape[1], p["idb"].data_ptr(), _lib.F32, idgb.data_ptr(), 2 * C,
                                        ws.data_ptr(), ws.numel(), s), "AADLayer id projection")
        out = torch.empty(B, H, W, C, dtype=dt, device=dev)
        need = B * C * 8 + B * H * W * 4 + (64 << 20)
        if need > ws.numel():
            ws = torch.empty(need + (1 << 20), dtype=torch.uint8, device=dev)
        _lib.check(lib.ghost_aad_layer_nhwc(_lib.gdtype(dt), h.data_ptr(), C, za.data_ptr(), Ca, B, H, W, C, Ca,
                                            p["gbw"].data_ptr(), p["gbw"].shape[0], p["gbw"].shape[1],
                                            p["gbb"].data_ptr(), p["wh"].data_ptr(), p["bh"].data_ptr(),
                                            idgb.data_ptr(), 2 * C, 0.0 if relu else 1.0, out.data_ptr(), C,
                                            ws.data_ptr(), ws.numel(), s), "AADLayer")
        out = out.permute(0, 3, 1, 2)
        return out.to(torch.float16) if pdt == torch.float16 else out   # .half(): the reference's dtype


class _Container(nn.Sequential):
    def forward(self, *inputs):  # noqa: D401
        raise NotImplementedError(
            f"ghost_amd: {type(self).__name__} is executed as part of AEI_Net.forward on the MI355X path; "
            "per-module torch execution is not shipped")


class AddBlocksSequential(_Container):
    """AddBlocksSequential (AADLayer.py:40-50): parameter container."""


class AAD_ResBlk(nn.Module):
    """AAD_ResBlk(cin, cout, c_attr, c_id, num_blocks) (AADLayer.py:53-72); executed by AEI_Net.forward."""

    def __init__(self, cin, cout, c_attr, c_id, num_blocks):
        super().__init__()
        self.cin = cin
        self.cout = cout
        add_blocks = []
        for i in range(num_blocks):
            out = cin if i < (num_blocks - 1) else cout
            add_blocks.extend([AADLayer(cin, c_attr, c_id), nn.ReLU(inplace=True),
                               nn.Conv2d(cin, out, kernel_size=3, stride=1, padding=1, bias=False)])
        self.add_blocks = AddBlocksSequential(*add_blocks)
        if cin != cout:
            self.last_add_block = AddBlocksSequential(AADLayer(cin, c_attr, c_id), nn.ReLU(inplace=True),
                                                      nn.Conv2d(cin, cout, kernel_size=3, stride=1, padding=1,
                                                                bias=False))

    def forward(self, h, z_attr, z_id):
        raise NotImplementedError("ghost_amd: AAD_ResBlk runs inside AEI_Net.forward on the MI355X path")

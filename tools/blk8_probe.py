"""AADBlk8 teacher-forced gate numbers (tests/test_bf16_parity.py check_blocks, block 8) for A/B of kernel
variants: python tools/blk8_probe.py [backbone nb B st] ..., prints Y max/mean and u8 max / fraction of bytes
differing against the storage emulation."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import test_bf16_parity as T  # noqa: E402
from oracle import aei_ref  # noqa: E402

cases = [("linknet", 3, 64, "bf16"), ("unet", 2, 64, "bf16"), ("linknet", 3, 2, "bf16"), ("unet", 3, 2, "bf16")]
for backbone, nb, B, st in cases:
    rows = T.ROWS if B == 64 else list(range(B))
    r = T.run(backbone, nb, B, rows=rows, st=st)
    p, z = r["p"], r["z"]
    with aei_ref.storage(T.STORE[st]):
        yk = aei_ref.gen_block_bf16_storage(r["blocks"][6], r["attr"][7], z, p, backbone, nb, 8)
    t8 = torch.tanh(yk)
    dY = (r["Y"] - aei_ref._q(t8)).abs()
    du = np.abs(r["u8"].astype(np.int16) - aei_ref.y_to_u8_bgr(t8).astype(np.int16))
    print(f"{os.environ.get('GHOST_V5_FLAGS', '-')} {backbone}/{nb} B={B} {st}: Y max {float(dY.max()):.4f} mean "
          f"{float(dY.mean()):.2e}  u8 max {int(du.max())} frac {(du > 0).mean():.4f}", flush=True)

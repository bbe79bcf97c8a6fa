"""Generate the golden vectors in tests/golden/ by running the REFERENCE itself.

Run in the build container only (it needs /root/reference, which does not exist on
the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What it does
* imports ``network.AEI_Net`` / ``network.AADLayer`` from /root/reference
  (read-only; nothing is copied — only their outputs are stored);
* checks that the reference ``state_dict`` keys/shapes equal ``oracle.aei_ref.param_specs``;
* fills the weights with the deterministic key-hashed recipe (``oracle.aei_ref.make_weights``);
* runs the reference CPU fp32 forward on seeded inputs and stores inputs-by-seed,
  outputs and attr checksums as small ``.npz`` files;
* runs the reference ``faceshifter_batch`` (utils/inference/faceshifter_run.py) on
  transform_target_to_torch-normalised synthetic uint8 crops for the u8 pipeline vector.

Fixtures are data (inputs by seed + expected outputs); no reference source is stored.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
from oracle import aei_ref  # noqa: E402

ATTR_SAMPLE = 4096


def attr_summary(attr):
    out = {}
    for i, a in enumerate(attr, 1):
        a = a.detach().double()
        flat = a.reshape(-1)
        idx = np.linspace(0, flat.numel() - 1, ATTR_SAMPLE).astype(np.int64)
        out[f"attr{i}_shape"] = np.array(a.shape, dtype=np.int64)
        out[f"attr{i}_sum"] = np.array(float(flat.sum()))
        out[f"attr{i}_abssum"] = np.array(float(flat.abs().sum()))
        out[f"attr{i}_idx"] = idx
        out[f"attr{i}_sample"] = flat[idx].float().numpy()
    return out


def build_ref(backbone, num_blocks, c_id=512):
    from network.AEI_Net import AEI_Net
    G = AEI_Net(backbone, num_blocks=num_blocks, c_id=c_id).eval()
    specs = aei_ref.param_specs(backbone, num_blocks, c_id)
    sd = G.state_dict()
    ref_keys = [(k, tuple(v.shape)) for k, v in sd.items()]
    mine = [(k, tuple(s)) for k, s, _ in specs]
    assert ref_keys == mine, "oracle param_specs disagree with the reference state_dict"
    w = aei_ref.make_weights(specs)
    G.load_state_dict(w, strict=True)
    return G, w


def forward_case(name, backbone, num_blocks, batch, seed=7, pipeline=False):
    G, _ = build_ref(backbone, num_blocks)
    xt, z = aei_ref.make_inputs(batch, seed)
    t0 = time.time()
    with torch.no_grad():
        y, attr = G(xt, z)
    dt = time.time() - t0
    rec = {"backbone": np.array(backbone), "num_blocks": np.array(num_blocks), "batch": np.array(batch),
           "seed": np.array(seed), "Y": y.numpy().astype(np.float32)}
    rec.update(attr_summary(attr))
    if pipeline:
        # u8 pipeline: synthetic BGR crops -> transform_target_to_torch(half=False) -> faceshifter_batch
        spec = importlib.util.spec_from_file_location("ref_faceshifter_run",
                                                      os.path.join(REF, "utils/inference/faceshifter_run.py"))
        fr = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(fr)
        crops = aei_ref.make_u8_crops(batch, seed=0)
        target = aei_ref.transform_target(crops)          # restated core.py:13-26 (it calls .cuda())
        src = z[:1]                                          # one identity, broadcast by faceshifter_batch
        u8 = fr.faceshifter_batch(src, target, G)
        with torch.no_grad():
            ypipe, _ = G(target, torch.cat([src] * batch))
        rec["crops_seed"] = np.array(0)
        rec["U8"] = np.asarray(u8, dtype=np.uint8)
        rec["Ypipe"] = ypipe.numpy().astype(np.float32)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **rec)
    print(f"{name}: fwd {dt:.2f}s  mean|Y|={float(y.abs().mean()):.4f}")


def aad_cases():
    from network.AADLayer import AADLayer
    cases = [(1024, 1024, 2), (1024, 2048, 4), (512, 512, 8), (256, 128, 16), (128, 64, 32), (64, 64, 32), (32, 32, 16)]
    rec = {"cases": np.array(cases, dtype=np.int64)}
    for i, (c_x, c_a, n) in enumerate(cases):
        layer = AADLayer(c_x, c_a, 512).eval()
        specs = [(f"case{i}.{k}", tuple(v.shape), "lin_w" if k.startswith("fc") and k.endswith("weight")
                  else ("bias" if k.endswith("bias") else "conv")) for k, v in layer.state_dict().items()]
        w = aei_ref.make_weights(specs)
        layer.load_state_dict({k.split(".", 1)[1]: v for k, v in w.items()})
        g = np.random.Generator(np.random.PCG64(100 + i))
        h = torch.from_numpy((g.normal(0.5, 2.0, size=(2, c_x, n, n))).astype(np.float32))
        za = torch.from_numpy(g.normal(0, 1, size=(2, c_a, n, n)).astype(np.float32))
        zi = torch.from_numpy(g.normal(0, 1, size=(2, 512)).astype(np.float32))
        with torch.no_grad():
            out = layer(h, za, zi)
        rec[f"case{i}_out"] = out.numpy()
    np.savez_compressed(os.path.join(HERE, "aad_layer_cases.npz"), **rec)
    print("aad_layer_cases written")


def main():
    if not os.path.isdir(REF):
        raise SystemExit("reference not present: golden vectors are regenerated only in the build container")
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    torch.set_num_threads(os.cpu_count() or 8)
    jobs = {
        "aei_unet2_b2": lambda: forward_case("aei_unet2_b2", "unet", 2, 2, pipeline=True),
        "aei_linknet3_b2": lambda: forward_case("aei_linknet3_b2", "linknet", 3, 2, pipeline=True),
        "aei_unet1_b1": lambda: forward_case("aei_unet1_b1", "unet", 1, 1),
        "aei_unet3_b1": lambda: forward_case("aei_unet3_b1", "unet", 3, 1),
        "aei_resnet2_b1": lambda: forward_case("aei_resnet2_b1", "resnet", 2, 1),
        "aad_layer_cases": aad_cases,
    }
    only = [a for a in sys.argv[1:] if not a.startswith("-")]   # regenerate a subset by name
    for name, job in jobs.items():
        if not only or name in only:
            job()


if __name__ == "__main__":
    main()

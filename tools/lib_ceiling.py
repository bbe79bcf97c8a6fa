"""Library ceilings on this box for the generator's conv shapes (B = 64, bf16): hipBLASLt GEMM of the
im2col-equivalent size and MIOpen's channels_last conv2d, HIP-event timed (a yardstick for the
hand-written halo conv, not part of the product)."""
import torch
import torch.nn.functional as F

dev = torch.device("cuda:0")


def t(fn, it=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


for H, ci, co in [(256, 64, 64), (128, 128, 128), (64, 256, 256), (32, 512, 512), (16, 1024, 1024)]:
    M, K, N = 64 * H * H, 9 * ci, co
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
    us = t(lambda: a @ b)
    fl = 2.0 * M * N * K
    del a, b
    x = torch.randn(64, ci, H, H, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    w = torch.randn(co, ci, 3, 3, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    try:
        uc = t(lambda: F.conv2d(x, w, padding=1), 10)
    except Exception as ex:  # noqa: BLE001
        uc = float("nan")
    print(f"H={H:3d} {ci:4d}->{co:4d}: GEMM {M}x{N}x{K} {us:8.1f} us {fl / us / 1e6:7.1f} TF/s | "
          f"conv2d channels_last {uc:8.1f} us {fl / uc / 1e6:7.1f} TF/s", flush=True)

"""Timing probe: item-tower forward (K4m) over n catalogue items for d in argv."""
import sys
import time

import torch

sys.path.insert(0, "hybrid-als-twotower-recommender_amd")
from src.tt_engine import DeviceTwoTower  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
    ds = [int(x) for x in sys.argv[2:]] or [128]
    for d in ds:
        tt = DeviceTwoTower(4, n, 2651, 255, d, seed=1, device_init=True)
        g = torch.Generator(device="cuda").manual_seed(2)
        it = torch.arange(n, dtype=torch.int32, device="cuda")
        mn = torch.randint(0, 2651, (n,), device="cuda", generator=g, dtype=torch.int32)
        ct = torch.randint(0, 255, (n,), device="cuda", generator=g, dtype=torch.int32)
        nu = torch.rand((n, 2), device="cuda", generator=g)
        out = tt.item_vectors(it, mn, ct, nu)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 3
        e0.record()
        for _ in range(reps):
            tt.item_vectors(it, mn, ct, nu, out=out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        tf = 2.0 * (d + 32) * d * n / ms / 1e9
        print(f"d {d}: {ms:.2f} ms for {n} items = {n / ms / 1e6:.2f} G items/s, {tf:.1f} TFLOP/s "
              f"({tf / 157.3:.3f} of f32 MFMA peak)", flush=True)
        del tt, it, mn, ct, nu, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

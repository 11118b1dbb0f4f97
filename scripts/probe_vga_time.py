"""VGA global kernel time at 1000^2 (configs[2]) for A/B builds selected with DMX_LIB.

    DMX_LIB=depthmapx_amd/_lib_ab/<variant>/libdmx.so python scripts/probe_vga_time.py [--grid 1000] [--reps 1]
"""
import argparse
import hashlib
import time
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import depthmapx_amd as dmx  # noqa: E402
from bench import load_lines  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=1)
    a = ap.parse_args()
    import torch
    W = a.grid
    ctx = dmx.Context(0)
    pm = dmx.PointMap([0.0, 0.0, float(W), float(W)], load_lines(W, 50), 1.0)
    assert pm.make_points(0.5, 0.5)
    N = pm.info()["filled"]
    g = pm.make_graph(ctx)
    mk = ctx.last_timing()[0]
    out = torch.full((N, 7), -1.0, dtype=torch.float32, device="cuda:0")
    ts, walls = [], []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.time()
        g.vga_visual_global_device(out.data_ptr())
        torch.cuda.synchronize()
        walls.append(time.time() - t0)
        ts.append(ctx.last_timing()[1])
    st = ctx.last_stats()
    chk = float(out[:, 5].double().sum().item())
    digest = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
    env = {k: v for k, v in os.environ.items() if k.startswith("DMX_")}
    print(json.dumps({"lib": os.environ.get("DMX_LIB", "default"), "env": env, "grid": W, "mk_s": mk, "vga_s": ts,
                      "wall_s": walls, "phase_cycles": ctx.last_phase_cycles(), "checksum_col5": chk, "digest": digest,
                      "stats": {k: v for k, v in st.items() if k.startswith("vga")}}), flush=True)


if __name__ == "__main__":
    main()

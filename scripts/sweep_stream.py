"""Sweep the stream-K decode GEMM's tile shapes (mt = 16-row MFMA tiles per
workgroup row block, bn = output columns per workgroup, grid = resident
workgroups) against the library GEMM for the Qwen2-7B decode shapes at batch
M, timed inside hipGraphs on cold rotating weights (the gemm_dispatch_table
harness).  Prints the best plan per (shape, M) and its effective HBM TB/s."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from githubrepostorag_amd.ops import linear as L  # noqa: E402

SHAPES = {"qkv": (4608, 3584), "o_proj": (3584, 3584), "gate_up": (37888, 3584), "down": (3584, 18944),
          "lm_head": (152064, 3584)}


def time_fn(fn, reps=20, rounds=5):
    """GPU time per call inside a captured hipGraph (as the decode step runs
    it), median of `rounds` replays of `reps` calls (same harness as
    scripts/gemm_dispatch_table.py)."""
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()
        fn()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    out = []
    for _ in range(rounds):
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / reps * 1000)
    del g
    return statistics.median(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="64,96,128")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--plans", default="4x64,4x128,4x256,8x64,8x128,8x256")
    ap.add_argument("--grids", default="256,512")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    L.enable_tuned_gemms()
    dev = torch.device("cuda")
    res = {}
    for name in a.shapes.split(","):
        N, K = SHAPES[name]
        ncopy = max(2, min(12, (1 << 30) // (N * K * 2) + 1))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(ncopy)]
        it = {"i": 0}

        def nxt():
            it["i"] = (it["i"] + 1) % ncopy
            return ws[it["i"]]

        for M in map(int, a.M.split(",")):
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            ref = torch.nn.functional.linear(x.float(), ws[0].float())
            cand = {"library": lambda: torch.nn.functional.linear(x, nxt())}
            for p in a.plans.split(","):
                mt, bn = map(int, p.split("x"))
                for g in map(int, a.grids.split(",")):
                    plan = (mt, bn, g)
                    y = L.gemm_stream(x, ws[0], None, plan=plan).float()
                    err = (y - ref).abs().max().item() / ref.abs().max().item()
                    assert err < 2e-2, (name, M, plan, err)
                    cand[f"stream_{mt}x{bn}_g{g}"] = (lambda pl=plan: L.gemm_stream(x, nxt(), None, plan=pl))
            t = {k: time_fn(f) for k, f in cand.items()}
            best = min(t, key=t.get)
            gb = N * K * 2 / 1e9
            res[f"{name}_M{M}"] = {k: round(v, 2) for k, v in t.items()}
            print(f"{name:8s} M={M:4d} library {t['library']:7.1f} us | best {best} {t[best]:7.1f} us "
                  f"({gb / (t[best] * 1e-6) / 1e3:.2f} TB/s)", flush=True)
            print("    " + " ".join(f"{k[7:]}={v:.1f}" for k, v in t.items() if k != "library"), flush=True)
        del ws
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

"""Decode-GEMM sweep: hipBLASLt vs the skinny kernel vs the split-K stream
kernel (auto plan + a plan grid), cold weights (rotating copies > MALL),
interleaved rounds in one process (cdna guide §5.4 rule 24)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from githubrepostorag_amd.ops.linear import gemm_skinny, gemm_stream, linear, stream_plan  # noqa: E402
from scripts.microbench import rounds  # noqa: E402

SHAPES = {"qkv": (4608, 3584), "o_proj": (3584, 3584), "gate_up": (37888, 3584), "down": (3584, 18944),
          "lm_head": (152064, 3584)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="32,64,128")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--sweep", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    out = {}
    for M in map(int, a.M.split(",")):
        for name in a.shapes.split(","):
            N, K = SHAPES[name]
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            ncopy = max(2, min(16, (1 << 30) // (N * K * 2) + 1))
            ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(ncopy)]
            it = {"i": 0}

            def nxt():
                it["i"] = (it["i"] + 1) % ncopy
                return ws[it["i"]]

            ref = torch.nn.functional.linear(x, ws[0]).float()
            var = {"hipblaslt": lambda: torch.nn.functional.linear(x, nxt()),
                   "stream_auto": lambda: gemm_stream(x, nxt()),
                   "dispatch": lambda: linear(x, nxt())}
            if M <= 64:
                var["skinny"] = lambda: gemm_skinny(x, nxt())
            plans = []
            if a.sweep:
                mt = 2 if M <= 32 else 4
                for bn in (128, 256):
                    plans.append((mt, bn, 256))
            for p in plans:
                var[f"stream_{p[0]}x{p[1]}s{p[2]}"] = (lambda p=p: gemm_stream(x, nxt(), None, p))
            errs = {}
            for k, fn in var.items():
                it["i"] = ncopy - 1
                y = fn().float()
                errs[k] = float((y - ref).abs().max())
            r = rounds(var, n=5, iters=30)
            gb = N * K * 2 / 1e9
            for k in r:
                r[k]["TB_s"] = round(gb / (r[k]["min_us"] * 1e-6) / 1e3, 2)
                r[k]["maxerr"] = round(errs[k], 4)
            r["auto_plan"] = list(stream_plan(M, N, K))
            out[f"{name}_M{M}"] = r
            best = min((v["min_us"], k) for k, v in r.items() if isinstance(v, dict))
            print(f"{name}_M{M}: best {best[1]} {best[0]}us; hipblaslt {r['hipblaslt']['min_us']}us; "
                  f"auto {r['stream_auto']['min_us']}us plan {r['auto_plan']}", flush=True)
            del ws
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

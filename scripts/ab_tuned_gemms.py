"""A/B every TunableOp solution of a raw results file against hipBLASLt's
default heuristic on cold rotating weights (CUDA events, interleaved rounds)
and keep only the entries that win by >= --min-gain.  Output is the file the
engine loads read-only (utils/runtime.enable_tuned_gemms)."""
import argparse
import os
import re
import shutil
import statistics
import sys
import tempfile

ap = argparse.ArgumentParser()
ap.add_argument("--raw", default="githubrepostorag_amd/tuning/tunableop_raw.csv")
ap.add_argument("--out", default="githubrepostorag_amd/tuning/tunableop_gfx950.csv")
ap.add_argument("--min-gain", type=float, default=1.03)
a = ap.parse_args()
lines = open(a.raw).read().splitlines()
head = [ln for ln in lines if ln.startswith("Validator")]
entries = [ln for ln in lines if ln.startswith("GemmTunableOp") and ",Default," not in ln]
tmp = tempfile.mkdtemp()
for ln in entries:
    pass
# one single-entry file per candidate, loaded in turn
os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "0"
import torch  # noqa: E402

dev = torch.device("cuda")


def time_gemm(x, ws, reps=30, rounds=5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = []
    for _ in range(rounds):
        torch.nn.functional.linear(x, ws[0])
        torch.cuda.synchronize()
        s.record()
        for i in range(reps):
            torch.nn.functional.linear(x, ws[i % len(ws)])
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / reps * 1000)
    return statistics.median(out)


keep = []
for ln in entries:
    m = re.match(r"GemmTunableOp_BFloat16_TN,tn_(\d+)_(\d+)_(\d+)_", ln)
    N, M, K = map(int, m.groups())
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    nw = max(2, min(8, (768 << 20) // (N * K * 2) + 1))
    ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(nw)]
    f = os.path.join(tmp, f"one_{M}_{N}_{K}.csv")
    with open(f.replace(".csv", "0.csv"), "w") as fh:
        fh.write("\n".join(head + [ln]) + "\n")
    torch.cuda.tunable.enable(False)
    t_def = time_gemm(x, ws)
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(False)
    torch.cuda.tunable.read_file(f.replace(".csv", "0.csv"))
    t_tun = time_gemm(x, ws)
    torch.cuda.tunable.enable(False)
    gain = t_def / t_tun
    verdict = "KEEP" if gain >= a.min_gain else "drop"
    print(f"M={M:6d} N={N:6d} K={K:6d} default {t_def:9.1f} us  tuned {t_tun:9.1f} us  x{gain:.3f} {verdict}",
          flush=True)
    if gain >= a.min_gain:
        keep.append(ln)
    del x, ws
with open(a.out, "w") as fh:
    fh.write("\n".join(head + keep) + "\n")
shutil.rmtree(tmp, ignore_errors=True)
print(f"kept {len(keep)}/{len(entries)} -> {a.out}")

"""Time the query-embedding path (bge-large, 64 synthetic questions) per stage."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from githubrepostorag_amd.embed.service import Embedder  # noqa: E402
from githubrepostorag_amd.utils import synthetic  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    emb = Embedder.from_name("bge-large-en-v1.5", device="cuda", seed=2)
    qs = [synthetic.question(i) for i in range(n)]
    for it in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ids = emb.tokenize(qs, emb.cfg.query_prefix)
        t1 = time.perf_counter()
        v = emb.embed_ids(ids)
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        print(f"iter {it}: tokenize {1e3 * (t1 - t0):.2f} ms, enqueue {1e3 * (t2 - t1):.2f} ms, "
              f"gpu-drain {1e3 * (t3 - t2):.2f} ms, tokens {sum(map(len, ids))}", flush=True)


if __name__ == "__main__":
    main()

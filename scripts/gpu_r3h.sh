# A/B of two kernel-library builds on the decode-attention microbench (old = HEAD, new = working tree)
set -o pipefail
mkdir -p gpurun_out
L=githubrepostorag_amd/_lib/libgrag_kernels.so
cp $L /tmp/cur.so &&
cp scripts/dev/_attn_ab/old.so $L && timeout -k 10 200 python -u scripts/microbench.py --what decode > gpurun_out/mb_dec_old.json 2>&1 &&
cp scripts/dev/_attn_ab/new.so $L && timeout -k 10 200 python -u scripts/microbench.py --what decode > gpurun_out/mb_dec_new.json 2>&1 &&
cp scripts/dev/_attn_ab/old.so $L && timeout -k 10 200 python -u scripts/microbench.py --what decode > gpurun_out/mb_dec_old2.json 2>&1 &&
cp scripts/dev/_attn_ab/new.so $L && timeout -k 10 200 python -u scripts/microbench.py --what decode > gpurun_out/mb_dec_new2.json 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "paged" --timeout 120 --timeout-method thread > gpurun_out/pytest_r3h.log 2>&1; rc=$?; cp /tmp/cur.so $L; tail -2 gpurun_out/pytest_r3h.log; exit $rc

# A/B two kernel-library builds (scripts/dev/_ab/old.so = HEAD, new.so = working tree) on one box:
#   bash scripts/ab_lib.sh "<command writing JSON lines to stdout>" TAG [rounds]
# runs the command old/new alternately ROUNDS times (default 2) into gpurun_out/ab_TAG_{old,new}_i.log and
# restores the working-tree library afterwards.
set -o pipefail
mkdir -p gpurun_out
L=githubrepostorag_amd/_lib/libgrag_kernels.so
cp $L /tmp/cur_lib.so || exit 1
rc=0
for i in $(seq 1 ${3:-2}); do
  for v in old new; do
    cp scripts/dev/_ab/$v.so $L && timeout -k 10 300 bash -c "$1" > gpurun_out/ab_$2_${v}_$i.log 2>&1 || { rc=$?; break 2; }
  done
done
cp /tmp/cur_lib.so $L
exit $rc

set -o pipefail
mkdir -p gpurun_out/s3n
for rep in 1 2; do
for f in 0 1 2 4 1000; do
  RT_STEAL_FACTOR=$f RT_AMD_LIB=abl/librt_stealab.so timeout -k 10 200 python tools/variants.py --configs c3,c5d --variants 0 --rounds 3 2>/dev/null | sed "s/^/f$f /" >> gpurun_out/s3n/var.log || exit 1
  RT_STEAL_FACTOR=$f RT_AMD_LIB=abl/librt_stealab.so timeout -k 10 100 python tools/share_cost.py 2>/dev/null | sed "s/^/f$f /" >> gpurun_out/s3n/share.log || exit 1
done
done

#!/bin/bash
# A/B of the KB8 projection's math on the pose kernel (one gpurun call): the in-tree build, then
# variants patched in a scratch copy of the tree (device libm sincos / atan2 / atan2f in place of the
# exact_math.h / glibc_math.h functions).  Timing only: the variants are not the product.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03kb8ab
mkdir -p $OUT
timeout -k 10 120 python $R/tools/pose_bench.py > $OUT/A_exact.jsonl 2>&1 || exit 1
for v in B_sincos C_atan2 D_all; do
  rm -rf /tmp/ab && cp -r $R /tmp/ab && cd /tmp/ab || exit 1
  F=orb_slam3_comments_ghr_amd/csrc/ba_common.h
  case $v in
    B_sincos) sed -i 's/osgx::sincos_psi(psi, sp, cp);/sincos(psi, \&sp, \&cp);/' $F ;;
    C_atan2) sed -i 's/osgx::atan2_rn(r, v\[2\])/atan2(r, v[2])/' $F ;;
    D_all) sed -i 's/osgx::sincos_psi(psi, sp, cp);/sincos(psi, \&sp, \&cp);/; s/osgx::atan2_rn(r, v\[2\])/atan2(r, v[2])/; s/osgm::atan2f_fd(/atan2f(/g' $F ;;
  esac
  grep -c "osgx::sincos_psi\|osgx::atan2_rn\|osgm::atan2f_fd" $F > $OUT/$v.grep
  make -j16 > $OUT/$v.build 2>&1 || exit 1
  timeout -k 10 120 python tools/pose_bench.py > $OUT/$v.jsonl 2>&1 || exit 1
  cd $R
done
echo done

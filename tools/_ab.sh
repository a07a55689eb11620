# A/B: liblgx.so vs the libraries named in $@ (tools/*.so), C5 probe shape, alternating
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/ab.txt
: > $OUT
for i in 1 2; do
for L in factors_of_serendipity_recommendation_amd/liblgx.so "$@"; do
LGX_LIB=$L ABL_B=${ABL_B:-131072} timeout -k 10 200 python -u tools/score_ablation.py 2>&1 | grep -v amdgpu.ids >> $OUT || exit 1
done; done

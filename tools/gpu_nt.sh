set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/nt.txt
for r in 1 2; do
timeout -k 10 200 python -u tools/nt_probe.py >> gpurun_out/nt.txt 2>&1 || { cat gpurun_out/nt.txt; exit 1; }
timeout -k 10 200 python -u tools/nt_probe.py --lib tools/liblgx_nt.so >> gpurun_out/nt.txt 2>&1 || { cat gpurun_out/nt.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/nt.txt

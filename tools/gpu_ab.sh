set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/ab.txt
for r in 1 2; do
for b in score_lab score_lab_eager; do
  echo "== $b" >> gpurun_out/ab.txt
  timeout -k 10 200 tools/$b 131072 >> gpurun_out/ab.txt 2>&1 || { cat gpurun_out/ab.txt; exit 1; }
done
done
cat gpurun_out/ab.txt

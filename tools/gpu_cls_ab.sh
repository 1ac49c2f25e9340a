set -o pipefail
A="--config c2id --steps 10 --warmup 3 --no-cpu-baseline --no-pcie --no-fastq --no-e2e --no-side-configs"
for v in base cls1 cls2 cls3; do
  if [ $v = base ]; then L=""; else L="GANON_HIP_LIB=genomeanonymizer_amd/variants/libganon_hip_$v.so"; fi
  env $L timeout -k 10 300 python bench.py $A > gpurun_out/cls_$v.json 2> gpurun_out/cls_$v.err || exit 1
  echo "$v done"
done

# PMC step summaries of the c3 / c5 side-config lines (bench.py reads profiles/r03/pmc_step_<config>.json for their traffic field).
set -o pipefail
TAG=r03c3 BENCH_ARGS="--config c3 --reads 10000000 --genome 25000000 --windows 2500 --germline 25000 --no-fastq --no-pcie --no-side-configs --no-e2e" bash tools/gpu_pmc_step.sh && \
python3 tools/pmc_step.py r03c3 c3 10000000 gpurun_out/pmc_step_c3.json && \
TAG=r03c5 BENCH_ARGS="--config c5 --reads 10000 --genome 100000000 --no-fastq --no-pcie --no-side-configs --no-e2e" bash tools/gpu_pmc_step.sh && \
python3 tools/pmc_step.py r03c5 c5 10000 gpurun_out/pmc_step_c5.json && echo ALLDONE

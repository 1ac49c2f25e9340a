# GPU A/B sequence: the gpu tests of test_indels + test_gpu, then c3 / c5 (side-config sizes) and c2 bench lines with per-kernel times. Each GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_indels.py tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
for c in c3 c5; do
  if [ $c = c3 ]; then A="--reads 10000000 --genome 25000000 --windows 2500 --germline 25000 --steps 10 --warmup 3"; else A="--reads 10000 --genome 100000000 --steps 5 --warmup 2"; fi
  timeout -k 10 400 python bench.py --config $c $A --no-side-configs > gpurun_out/ab_$c.json 2> gpurun_out/ab_$c.err || { tail -20 gpurun_out/ab_$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$c.json'));print('$c', d['ms_per_step'], {k:v['avg_ms'] for k,v in d['pass']['kernels'].items()})"
done
timeout -k 10 400 python bench.py --steps 50 --warmup 10 --no-side-configs > gpurun_out/ab_c2.json 2> gpurun_out/ab_c2.err || { tail -20 gpurun_out/ab_c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/ab_c2.json'));print('c2', d['ms_per_step'], d['one_stream_ms_per_step'], {k:v['avg_ms'] for k,v in d['pass']['kernels'].items()})"
echo exit=0

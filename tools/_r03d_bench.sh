set -e
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03d_bench.json 2> gpurun_out/r03d_bench.err
for s in 20000:25000 10000:12500 5000:6250; do
  n=${s%%:*}; e=${s##*:}
  timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --total-samples $n --expert-rows $e --no-cpu-baseline > gpurun_out/r03d_share_${n}.json 2>> gpurun_out/r03d_bench.err
done

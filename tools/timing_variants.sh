set -e
for t in dispatch bracket both; do
  timeout -k 10 120 python bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-cold --compute-us 0 --timing $t > gpurun_out/tv_$t.log 2>&1
done
timeout -k 10 120 python bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-cold --compute-us 0 --sample-every 100000 > gpurun_out/tv_none.log 2>&1
timeout -k 10 120 python bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-cold --compute-us 0 --timing dispatch --sample-every 1 > gpurun_out/tv_all.log 2>&1

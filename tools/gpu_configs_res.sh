#!/bin/bash
# Resident learners (the bench's default form): BASELINE configs[2..4] at their own sizes and
# settings on one GPU (two co-resident learners, batched), the f1 trainer in both loop orders
# (the reference's: write-through; resident: update_send, update_wait, step) and the host cost
# per round of every form.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_configs_res.sh <tag>
set -o pipefail
TAG=${1:-cfgres}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/host_overhead.py > gpurun_out/${TAG}_host.json 2> gpurun_out/${TAG}_host.err \
    || { echo "host overhead failed"; tail gpurun_out/${TAG}_host.err; exit 1; }
cat gpurun_out/${TAG}_host.json
B="--steps 50 --warmup 10 --no-cpu-baseline --no-sweep"
run() {
  name=$1; shift
  timeout -k 10 600 python3 bench.py $B "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err \
      || { echo "$name failed"; tail gpurun_out/${TAG}_$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$name.json'));r=d['roofline'];print('$name','value',d['value'],'ms',d['ms_per_step'],'avg',d['averagings'],'cold',r['frac'],'inloop',r['in_loop']['frac'],'sec',d.get('secondary_publish',{}).get('value'),'parity',d['parity_of_timed_transport'])"
}
run 100m_clock --numel 100000000 --interpolation clock
run 1b_bf16_loss_decay --numel 1000000000 --dtype bf16 --interpolation loss --divergence-threshold 0.5 --loss-schedule decay
run 7b_bf16_p07 --numel 7000000000 --dtype bf16 --fetch-probability 0.7
for b in 8 128; do
  for form in "" "--resident"; do
    f=${form:+_resident}
    timeout -k 10 300 python3 examples/resnet18_gossip.py --learners 2 --steps 60 --batch-size $b $form \
        > gpurun_out/${TAG}_resnet18_b$b$f.json 2> gpurun_out/${TAG}_resnet18_b$b$f.err || { echo "resnet b$b$f failed"; tail gpurun_out/${TAG}_resnet18_b$b$f.err; exit 1; }
    cat gpurun_out/${TAG}_resnet18_b$b$f.json
  done
done
echo done

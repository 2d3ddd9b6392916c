# windows-per-UNet-call sweep of the bench workload (configs[1]), two alternated rounds
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for w in ${WPB_LIST:-32 48 24}; do
    timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-single-window --no-whisper --windows-per-batch $w > gpurun_out/wpb_$w.log 2>&1 || exit 1
    echo "r$r wpb=$w $(tail -1 gpurun_out/wpb_$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/wpb_sweep.log
  done
done

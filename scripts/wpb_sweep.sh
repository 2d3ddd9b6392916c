# windows-per-batch sweep (configs[1] 16/24/32, configs[4] 2/4): same box, no CPU baseline
set -o pipefail
mkdir -p gpurun_out
for w in 16 24 32; do
  timeout -k 10 300 python -u bench.py --windows-per-batch $w --steps 2 --no-cpu-baseline --no-single-window --no-whisper 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg1 w=$w', d['value'], d['ms_per_step'])" || exit 1
done
for w in 2 4; do
  timeout -k 10 300 python -u bench.py --config 4 --windows-per-batch $w --steps 2 --no-cpu-baseline --no-single-window --no-whisper 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg4 w=$w', d['value'], d['ms_per_step'])" || exit 1
done

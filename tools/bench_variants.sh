set -e
for a in "--steps 20 --warmup 5" "--steps 20 --warmup 5 --event-every 0" "--steps 200 --warmup 20" "--steps 200 --warmup 20 --event-every 0" "--steps 200 --warmup 2000" "--steps 200 --warmup 2000 --event-every 0" "--steps 20 --warmup 5"; do
  timeout -k 10 120 python bench.py --no-extras --no-cpu-baseline $a > /tmp/b.json
  python -c "import json;d=json.load(open('/tmp/b.json'));print('$a', d['ms_per_step']*1000, 'us/step', d['kernel_ms_per_launch']*1000, d.get('kernel_ms_sampled_events'))"
done

set -e
mkdir -p gpurun_out/c4
timeout -k 10 600 python -u bench.py --workload c4 --steps 1 --warmup 1 --cpu-baseline off > gpurun_out/c4/c4.json 2> gpurun_out/c4/c4.err
python -c "import json; d=json.load(open('gpurun_out/c4/c4.json')); print('c4', round(d['value']), round(d['kernel_ms_avg'],1), d['config'], d['occupancy']['lds_bytes_per_wg'])"
timeout -k 10 300 python -u bench.py --workload c2 --steps 2 --warmup 1 --cpu-baseline off > gpurun_out/c4/c2.json 2> gpurun_out/c4/c2.err
python -c "import json; d=json.load(open('gpurun_out/c4/c2.json')); print('c2', round(d['value']), round(d['kernel_ms_avg'],1))"

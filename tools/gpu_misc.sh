set -e
mkdir -p gpurun_out/v1618
timeout -k 10 300 python -u tools/ab.py --variants 16 18 --rounds 3 --grid 11 --persistent > gpurun_out/v1618/g11.txt 2>&1
tail -3 gpurun_out/v1618/g11.txt
timeout -k 10 300 python -u tools/ab.py --variants 16 18 --rounds 3 --grid 16 --persistent > gpurun_out/v1618/g16.txt 2>&1
tail -3 gpurun_out/v1618/g16.txt
timeout -k 10 600 python -u bench.py --workload c4 --steps 1 --warmup 1 --cpu-baseline off > gpurun_out/v1618/c4.json 2> gpurun_out/v1618/c4.err
python -c "import json; d=json.load(open('gpurun_out/v1618/c4.json')); print('c4', round(d['value']), round(d['kernel_ms_avg'],1), d['occupancy'])"

set -e
mkdir -p gpurun_out/c4p
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4p/prof -o prof -- python3 bench.py --workload c4 --steps 1 --warmup 1 --cpu-baseline off > gpurun_out/c4p/bench.json 2> gpurun_out/c4p/prof.err
PMC_PASSES="waves insts fetch write" profiles/pmc.sh gpurun_out/c4p/pmc --workload c4 --steps 1 --warmup 1

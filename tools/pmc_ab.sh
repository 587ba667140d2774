mkdir -p gpurun_out
PMC_PASSES="waves insts sched" bash profiles/pmc.sh gpurun_out/pmc_v5 --variant 5 --lpp 4
PMC_PASSES="waves insts sched" bash profiles/pmc.sh gpurun_out/pmc_v9 --variant 9 --lpp 4

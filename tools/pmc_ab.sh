mkdir -p gpurun_out
PMC_PASSES="waves insts lds" bash profiles/pmc.sh gpurun_out/pmc_v11 --variant 11 --lpp 4

mkdir -p gpurun_out
PMC_PASSES="waves insts lds fetch write" bash profiles/pmc.sh gpurun_out/pmc_v11b

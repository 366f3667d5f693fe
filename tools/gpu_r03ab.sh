# k_combined counters, lock-step (base) vs flat sweep (variant f)
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_WAVES SQ_ACTIVE_INST_SCA"
P3="TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
bash tools/pmc.sh r03ab_base "$P1" "$P2" "$P3" && \
GWAOI_LIB=$PWD/goworld_amd/lib/variants/f.so bash tools/pmc.sh r03ab_flat "$P1" "$P2" "$P3" && \
for t in base flat; do echo "== $t"; python3 tools/pmc_median.py gpurun_out/pmc_r03ab_$t k_combined; done > gpurun_out/pmc_r03ab.txt
cat gpurun_out/pmc_r03ab.txt

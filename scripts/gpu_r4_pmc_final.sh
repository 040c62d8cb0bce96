#!/bin/bash
# SQ counter passes of the final x6n table kernel, standalone 512-column blocks at D = H = 64 and 128
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r4pmcfinal}
mkdir -p $out
export PMC_SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE|SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU|SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM"
timeout -k 10 300 python scripts/bench_table.py --blocks 8 --rounds 3 > $out/table64.txt 2>&1 || { tail -5 $out/table64.txt; exit 1; }
grep "ms/block" $out/table64.txt
timeout -k 10 300 python scripts/bench_table.py --dim 128 --hidden 128 --blocks 4 --rounds 3 > $out/table128.txt 2>&1 || { tail -5 $out/table128.txt; exit 1; }
grep "ms/block" $out/table128.txt
timeout -k 10 600 scripts/gpu_pmc_cmd.sh r4final_x6n64 x6n_kernel scripts/bench_table.py --blocks 8 --rounds 1 > $out/pmc64.txt 2>&1 || { tail -5 $out/pmc64.txt; exit 1; }
timeout -k 10 600 scripts/gpu_pmc_cmd.sh r4final_x6n128 x6n_kernel scripts/bench_table.py --dim 128 --hidden 128 --blocks 4 --rounds 1 > $out/pmc128.txt 2>&1 || { tail -5 $out/pmc128.txt; exit 1; }
echo done

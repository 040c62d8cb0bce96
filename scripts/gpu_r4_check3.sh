#!/bin/bash
# GPU suite + bench after the gather fix, then the round-4 SQ counter passes of the pair-table kernel
# (standalone 512-column blocks at config-4 geometry, scripts/bench_table.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r4check3}
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail=10 -q -rf --durations=15 --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/pytest_gpu.log
tail -6 $out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cut -c1-200 $out/bench.json
timeout -k 10 300 python scripts/bench_table.py --blocks 8 --rounds 3 > $out/table_alone.txt 2>&1 || { tail -5 $out/table_alone.txt; exit 1; }
tail -2 $out/table_alone.txt
export PMC_SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE|SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU|SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM"
timeout -k 10 600 scripts/gpu_pmc_cmd.sh r4table_x6n x6n_kernel scripts/bench_table.py --blocks 8 --rounds 1 > $out/pmc.txt 2>&1 || { tail -5 $out/pmc.txt; exit 1; }
tail -20 $out/pmc.txt
NAIS_X6N=0 timeout -k 10 600 scripts/gpu_pmc_cmd.sh r4table_x3b x3b_kernel scripts/bench_table.py --blocks 8 --rounds 1 > $out/pmc_x3b.txt 2>&1 || { tail -5 $out/pmc_x3b.txt; exit 1; }
tail -20 $out/pmc_x3b.txt
timeout -k 10 300 python scripts/bench_table.py --dim 128 --hidden 128 --blocks 4 --rounds 3 > $out/table128_alone.txt 2>&1 || { tail -5 $out/table128_alone.txt; exit 1; }
tail -2 $out/table128_alone.txt
timeout -k 10 600 scripts/gpu_pmc_cmd.sh r4table_x6n128 x6n_kernel scripts/bench_table.py --dim 128 --hidden 128 --blocks 4 --rounds 1 > $out/pmc128.txt 2>&1 || { tail -5 $out/pmc128.txt; exit 1; }
tail -20 $out/pmc128.txt

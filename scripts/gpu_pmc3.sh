set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1

NAIS_HIP_LIB=$GRAFT_REPO_ROOT/build_ab/nobuild.so timeout -k 10 600 scripts/gpu_pmc_cmd.sh r5nobuild x6n_kernel scripts/bench_table.py --blocks 8 --rounds 1 > gpurun_out/pmc_nobuild.txt 2>&1 || { tail -5 gpurun_out/pmc_nobuild.txt; exit 1; }
timeout -k 10 600 scripts/gpu_pmc_cmd.sh r5rd x6n_kernel scripts/bench_table.py --blocks 8 --rounds 1 --variant region_distance > gpurun_out/pmc_rd.txt 2>&1 || { tail -5 gpurun_out/pmc_rd.txt; exit 1; }
tail -22 gpurun_out/pmc_nobuild.txt; tail -22 gpurun_out/pmc_rd.txt

#!/bin/bash
# 4-block f32 MFMA distance term: layout probe, parity of the variant library on the distance
# tests, then the region_distance table block A/B (in-tree vs build_ab/d4b.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r5d4b
mkdir -p $out
timeout -k 5 60 ./build_ab/mbx > $out/mfma_4b_layout.txt 2>&1 || exit 1
NAIS_HIP_LIB=build_ab/d4b.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_any_shape.py -m gpu -q -x -k "distance" --timeout 300 --timeout-method thread > $out/pytest_d4b.log 2>&1
rc=$?; tail -3 $out/pytest_d4b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_table.py --blocks 8 --rounds 4 --variant region_distance --lib d4b=build_ab/d4b.so --lib d4bc=build_ab/d4bc.so > $out/rd64.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_table.py --blocks 4 --rounds 3 --dim 128 --hidden 128 --variant region_distance --lib d4b=build_ab/d4b.so --lib d4bc=build_ab/d4bc.so > $out/rd128.txt 2>&1 || exit 1
grep -h "ms/block" $out/rd64.txt $out/rd128.txt

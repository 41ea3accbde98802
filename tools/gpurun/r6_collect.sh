#!/bin/bash
# round 6 (container side, after r6_evidence.sh): copy the evidence into profiles/ under distinct names
set -e
cd "$(dirname "$0")/../.."
O=gpurun_out/r6ev
P=profiles/round6
cp $O/pytest.log ${P}_pytest_gpu.log
cp $O/smoke.log ${P}_smoke.log
cp $O/round6_msm_pmc_n65536.json $O/round6_msm_pmc_n2097152.json $O/round6_bls_pmc_n16384.json profiles/
cp $O/bls_trace/run_kernel_stats.csv ${P}_bls_leg_rocprof_kernel_stats.csv
cp $O/bench.json ${P}_final_bench.json
cp $O/bench_s20.json ${P}_bench_s20.json
cp $O/prof1/b_kernel_stats.csv ${P}_headline_inflight1_rocprof_kernel_stats.csv
cp $O/headline_inflight1_bench_line.json ${P}_headline_inflight1_bench_line.json
cp $O/prof12/b_kernel_stats.csv ${P}_headline_inflight12_rocprof_kernel_stats.csv
cp $O/headline_inflight12_bench_line.json ${P}_headline_inflight12_bench_line.json
echo collected

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for B in 1048576 131072; do
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d gpurun_out/envpmc_$B -o run -- python3 tools/bench_env.py $B 2 > gpurun_out/envpmc_$B.log 2>&1 || exit $?
done

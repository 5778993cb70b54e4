set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ldsb
timeout -k 10 60 ./tools/lds_bank_bench > gpurun_out/ldsb/times.txt 2>&1
cd /tmp && export TMPDIR=/tmp
for m in b32 u8 u16 b64 b32lp b64lp; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d $GRAFT_REPO_ROOT/gpurun_out/ldsb/pmc_$m -o pmc --output-format csv -- $GRAFT_REPO_ROOT/tools/lds_bank_bench 268435456 $m > $GRAFT_REPO_ROOT/gpurun_out/ldsb/pmc_$m.log 2>&1
done
echo done

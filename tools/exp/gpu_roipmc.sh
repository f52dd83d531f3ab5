# roi_align sweep kernel SQ counters, exact vs FMA (TRK_TUNE), one rocprofv3 pass each
set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
export TMPDIR=/tmp
for v in 0 1; do
  TRK_TUNE=roi_fma=$v timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/roipmc_$v -o run --output-format csv -- python3 tools/roi_only.py 5 > /dev/null 2>&1 || exit 1
done
echo done

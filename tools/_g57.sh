# round-5 GPU call 57: PMC of the three lm_head GEMMs at the final HEAD (planning data for round 6)
cd $GRAFT_REPO_ROOT
S="A SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
T="B TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE"
for l in nt nn tn; do
  PMC_SETS="$S;$T" bash tools/pmc_run.sh pmc57$l python3 $GRAFT_REPO_ROOT/tools/gemm4_probe.py --layouts $l --shapes lmhead --scheds 0 --rounds 1 --iters 3 || exit $?
  python3 tools/pmc_summary.py gpurun_out/pmc57$l > gpurun_out/sum_pmc57$l.txt; rm -rf gpurun_out/pmc57$l/*/
done
grep -h "MFMA busy" gpurun_out/sum_pmc57*.txt

cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python -u tools/gemm_tt_bench.py > gpurun_out/gtt_default.log 2>&1 && timeout -k 10 180 python -u tools/gemm_tt_bench.py torch > gpurun_out/gtt_torch.log 2>&1 || exit 1
for c in 1,256,512 2,256,512 3,256,512 4,256,512 5,256,512 7,256,512 2,128,1024 4,128,1024 3,128,1024 2,256,1024; do
  XRS_GEMM_CFG=$c timeout -k 10 120 python -u tools/gemm_tt_bench.py > gpurun_out/gtt_$c.log 2>&1 || exit 1
done

cd "${GRAFT_REPO_ROOT}"
for r in 16384 32768 65536 131072 262144 524288; do
  echo "ROWS=$r"; ROWS=$r SHAPE="wgrad M64 N64" timeout -k 10 60 python scripts/gemm_bench.py 2>/dev/null || exit 1
  ROWS=$r SHAPE="wgrad M64 N192" timeout -k 10 60 python scripts/gemm_bench.py 2>/dev/null || exit 1
done
for mc in 64 128 256 512 1024; do
  echo "MAXCHUNKS=$mc MINROWS=16"; DGPPO_WGRAD_MINROWS=16 DGPPO_WGRAD_MAXCHUNKS=$mc SHAPE="wgrad M64 N64" timeout -k 10 60 python scripts/gemm_bench.py 2>/dev/null || exit 1
done

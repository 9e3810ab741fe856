L=safe-dreamer_amd/sdreamer
mkdir -p gpurun_out/r05l
for i in 1 2; do
 for lib in _lib _lib_p0 _lib_w0; do
  SDHIP_LIB=$L/$lib/libsdhip.so timeout -k 10 120 python tools/mlp_bench.py 16384 2560 30 2>&1 | grep mlp | sed "s/^/$lib /" >> gpurun_out/r05l/mlp.txt || exit 1
 done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gemm.py -k "mlp or heads" > gpurun_out/r05l/tests.txt 2>&1

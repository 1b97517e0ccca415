set -u
timeout -k 10 600 python -u -m pytest tests/test_gatconv_gpu.py tests/test_bench_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/lg_tests.txt 2>&1
rc=$?; echo "pytest product rc=$rc"; tail -2 gpurun_out/lg_tests.txt; [ $rc -eq 0 ] || exit $rc
GFD_LIB_PATH=$PWD/gnn-fraud-detection_amd/gfd/libgfd_rot.so timeout -k 10 600 python -u -m pytest tests/test_gatconv_gpu.py tests/test_bench_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "not bf16 and not c5" > gpurun_out/lg_tests_rot.txt 2>&1
rc=$?; echo "pytest rot rc=$rc"; tail -2 gpurun_out/lg_tests_rot.txt; [ $rc -eq 0 ] || exit $rc
scripts/gpu_ab.sh base - rot base - rot

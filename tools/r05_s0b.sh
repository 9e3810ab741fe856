set -o pipefail
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_dreamer.py -k "graph or matches_reference" > $O/tests.txt 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/timeline.py 4 > $O/timeline.txt 2>&1 || exit 1
bash tools/ab_env.sh 3 "" "SDREAMER_SIDE_PREP=0" "SDREAMER_SIDE_PREP=2" > $O/ab.txt 2>&1 || exit 1

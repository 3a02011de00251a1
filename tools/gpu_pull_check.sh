set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r1
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/r1/gpu_tests.log 2>&1
timeout -k 10 400 python tools/ab_trace.py --rounds 6 --variant CRGC_PULL=0 --variant CRGC_PULL=1,CRGC_PULL_DIV=16 --variant CRGC_PULL=1,CRGC_PULL_DIV=4 --variant CRGC_PULL=1,CRGC_PULL_DIV=64 > gpurun_out/r1/ab_pull.json 2> gpurun_out/r1/ab_pull.err

set -o pipefail
mkdir -p gpurun_out
MBLS_LG16=1 MBLS_LG16_PREP=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/lg16_tests.log 2>&1 || { tail -40 gpurun_out/lg16_tests.log; exit 1; }
tail -2 gpurun_out/lg16_tests.log
SETTINGS="MBLS_LG16=1,MBLS_LG16_PREP=1 MBLS_LG16=1 -" WORKLOADS="mainnet_block epoch_replay_cold" STEPS=20 bash tools/ab_env.sh

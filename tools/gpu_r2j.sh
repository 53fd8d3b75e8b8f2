set -e -o pipefail
bash tools/gpu_quick.sh r2j
mkdir -p gpurun_out/r2j
DQ_HIP_TRACE=1 timeout -k 10 120 python -u tools/c4_host.py 4 > gpurun_out/r2j/c4_host.out 2> gpurun_out/r2j/c4_host.err

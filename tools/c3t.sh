set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/c3t2
DQ_HIP_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/c3t2/prof -o run -- python3 -u tools/c3_trace.py 10 > gpurun_out/c3t2/calls.txt 2> gpurun_out/c3t2/host.txt
python3 tools/timeline.py gpurun_out/c3t2/prof 130 > gpurun_out/c3t2/timeline.txt
DQ_HIP_TRACE=1 timeout -k 10 300 python3 -u tools/c3_trace.py 10 > gpurun_out/c3t2/calls_noprof.txt 2> gpurun_out/c3t2/host_noprof.txt
echo ok

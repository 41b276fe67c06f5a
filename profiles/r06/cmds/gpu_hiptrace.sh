# HIP API durations of a 1-thread device-update queue run (which HIP call the worker's launch spends its time in)
set -o pipefail
O=gpurun_out/hiptrace
mkdir -p $O
make -s -C tests/c queue_bench || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --stats --output-format csv -d $O/t1 -o run -- build/ctest/queue_bench 131072 1 devupdate 1024 > $O/t1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --stats --output-format csv -d $O/t16 -o run -- build/ctest/queue_bench 131072 16 devupdate 64 > $O/t16.log 2>&1 || exit 1
find $O -name "*stats*.csv" | head

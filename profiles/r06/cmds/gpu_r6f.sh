# queue timeline: roctx markers + HIP runtime API + kernels for device-cell encode and update queues
set -o pipefail
mkdir -p gpurun_out/r6f
make -s -C tests/c queue_bench || exit 1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --hip-runtime-trace -d gpurun_out/r6f/enc -o q -- build/ctest/queue_bench 131072 16 device 64 > gpurun_out/r6f/enc.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --hip-runtime-trace -d gpurun_out/r6f/upd -o q -- build/ctest/queue_bench 131072 16 devupdate 64 > gpurun_out/r6f/upd.log 2>&1 || exit 1
echo ALLDONE

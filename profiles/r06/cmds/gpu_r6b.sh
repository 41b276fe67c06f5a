set -o pipefail
mkdir -p gpurun_out/r6b
make -s -C tests/c queue_bench dropin_bench || exit 1
timeout -k 10 180 python -u tools/short_launch.py > gpurun_out/r6b/short_launch.log 2>&1 || exit 1
for isa in avx512-gfni avx2 scalar; do
  ECG_CPU_ISA=$isa timeout -k 10 300 build/ctest/dropin_bench 4194304 > gpurun_out/r6b/dropin_$isa.log 2>&1 || exit 1
done
QB_VERIFY=1 timeout -k 10 120 build/ctest/queue_bench 131072 16 devupdate 16 > gpurun_out/r6b/qb_devupdate_verify.log 2>&1 || exit 1
for C in 131072 1048576; do
  timeout -k 10 300 build/ctest/queue_bench $C 16 devupdate 64 >> gpurun_out/r6b/qb_devupdate.log 2>&1 || exit 1
done
QB_CPU_QUEUE=1 timeout -k 10 300 build/ctest/queue_bench 131072 16 update 32 > gpurun_out/r6b/qb_cpuqueue.log 2>&1 || exit 1
QB_CPU_QUEUE=1 timeout -k 10 300 build/ctest/queue_bench 131072 16 > gpurun_out/r6b/qb_cpuqueue_encode.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6b/prof_short -o short -- python3 -u tools/short_launch.py --reps 50 > gpurun_out/r6b/short_launch_rocprof.log 2>&1 || exit 1
echo ALLDONE

# worker poll interval of device batches in flight: 20 us (product) vs 10 / 5 us (ab_p10000/, ab_p5000/),
# interleaved, 3 rounds: one-request latency and 16-thread throughput, device cells
set -o pipefail
O=gpurun_out/poll_ab
mkdir -p $O
make -s -C tests/c queue_bench || exit 1
for rep in 1 2 3; do
  for lib in p20000 p10000 p5000; do
    L=""; [ $lib != p20000 ] && L=ab_$lib
    for mode in device devupdate; do
      echo "== $lib $mode latency" >> $O/ab.log
      QB_LATENCY=1 LD_LIBRARY_PATH=$L timeout -k 10 120 build/ctest/queue_bench 131072 1 $mode 64 2>/dev/null | grep '^{' >> $O/ab.log || exit 1
      echo "== $lib $mode T=16" >> $O/ab.log
      LD_LIBRARY_PATH=$L timeout -k 10 120 build/ctest/queue_bench 131072 16 $mode 64 2>/dev/null | grep '^{' >> $O/ab.log || exit 1
    done
  done
done
cat $O/ab.log

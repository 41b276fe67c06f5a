# host-cell queue A/B in one process pool: the committed early-close rule (product lib) vs no early close (ab_old/,
# built from 40291be), interleaved, 3 rounds; throughput and one-request latency
set -o pipefail
O=gpurun_out/qhost_ab
mkdir -p $O
make -s -C tests/c queue_bench || exit 1
for rep in 1 2 3; do
  for lib in new old; do
    L=""; [ $lib = old ] && L=ab_old
    for C in 131072 1048576; do
      for T in 1 16; do
        echo "== $lib C=$C T=$T" >> $O/ab.log
        LD_LIBRARY_PATH=$L timeout -k 10 120 build/ctest/queue_bench $C $T 2>/dev/null | grep '^{' >> $O/ab.log || exit 1
      done
      echo "== $lib C=$C latency" >> $O/ab.log
      QB_LATENCY=1 LD_LIBRARY_PATH=$L timeout -k 10 120 build/ctest/queue_bench $C 1 2>/dev/null | grep '^{' >> $O/ab.log || exit 1
    done
  done
done
cat $O/ab.log

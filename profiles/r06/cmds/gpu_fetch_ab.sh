# table upload A/B on large device-cell batches: fetch kernel (qt_tmp/) vs hipMemcpyAsync (qt8/), 1 MiB / 128 KiB cells
set -o pipefail
O=gpurun_out/fetch_ab
mkdir -p $O
make -s -C tests/c queue_bench || exit 1
for rep in 1 2 3; do
  for lib in qt_tmp qt8; do
    for C in 1048576 131072; do
      for T in 1 16; do
        echo "== $lib C=$C T=$T" >> $O/ab.log
        LD_LIBRARY_PATH=$lib timeout -k 10 300 build/ctest/queue_bench $C $T device $((1024 / T)) 2>/dev/null | grep '^{' >> $O/ab.log || exit 1
      done
    done
  done
done
cat $O/ab.log

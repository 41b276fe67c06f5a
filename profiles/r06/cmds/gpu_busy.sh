# host cost of one batched call on an idle vs a busy stream (fetch-kernel build vs -DECG_TABLE_MEMCPY in qt8/)
set -o pipefail
O=gpurun_out/busy
mkdir -p $O
make -s -C tests/c upd_latency || exit 1
timeout -k 10 120 build/ctest/upd_latency > $O/upd_latency.log 2>&1 || exit 1
LD_LIBRARY_PATH=qt8 timeout -k 10 120 build/ctest/upd_latency > $O/upd_latency_memcpy.log 2>&1 || exit 1
cat $O/*.log

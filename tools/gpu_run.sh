#!/bin/bash
# GPU-box driver for one gpurun call.  Every GPU step has its own time limit;
# any fault / abort / segfault / timeout ends the call (no retries).  Test
# failures (pytest exit 1) are not faults and do not stop later steps.
#   tools/gpu_run.sh [smoke] [tests] [bench] [prof] [pmc] [pmcjson] [rehearse8] [ecab] [exptests] ...
# Output: gpurun_out/<step>.log (OUT=subdir puts everything under gpurun_out/$OUT).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out${OUT:+/$OUT}
mkdir -p "$O"
export TMPDIR=/tmp

step() {   # name timeout cmd...
	local name=$1 to=$2
	shift 2
	echo "== $name: $*"
	timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
	local rc=$?
	echo "== $name rc=$rc"
	tail -n 12 "$O/$name.log"
	return $rc
}

PYTEST="python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread"

for what in "$@"; do
	case $what in
	smoke)
		step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
		;;
	tests)            # the whole GPU suite, as the driver runs it at round end
		step pytest_gpu 1100 $PYTEST tests -m gpu
		rc=$?; [ $rc -le 1 ] || exit $rc
		;;
	bench)
		step bench 900 python bench.py || exit $?
		;;
	prof)             # kernel trace + stats of the headline (profiles/rNN/rocprof_stats)
		rm -rf "$O/prof"
		step rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run \
			-- python3 bench.py --steps 10 --warmup 2 --no-detail --no-cpu || exit $?
		;;
	pmc)              # HBM bytes of the headline kernel: FETCH_SIZE and WRITE_SIZE passes
		rm -rf "$O/pmc_fetch" "$O/pmc_write"
		step rocprof_fetch 300 timeout -s KILL 280 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv \
			-d "$O/pmc_fetch" -o run -- python3 bench.py --steps 4 --warmup 1 --no-detail --no-cpu --profile-only \
			|| exit $?
		step rocprof_write 300 timeout -s KILL 280 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv \
			-d "$O/pmc_write" -o run -- python3 bench.py --steps 4 --warmup 1 --no-detail --no-cpu --profile-only \
			|| exit $?
		python tools/pmc_traffic.py "$O/pmc_fetch" "$O/pmc_write" "ecg_mm_kernel<4, 2" 6442450944 \
			"$O/pmc_traffic.json" || exit $?
		;;
	ecpmc)            # HBM bytes of the wide shapes (EC_8P2 decode, EC_16P2 encode / decode)
		for w in dec_8p2 enc_16p2 dec_16p2; do
			rm -rf "$O/pmc_${w}_f" "$O/pmc_${w}_w"
			step rocprof_${w}_f 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv \
				-d "$O/pmc_${w}_f" -o run -- python3 tools/ec_pmc.py $w || exit $?
			step rocprof_${w}_w 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv \
				-d "$O/pmc_${w}_w" -o run -- python3 tools/ec_pmc.py $w || exit $?
		done
		python tools/pmc_traffic.py "$O/pmc_dec_8p2_f" "$O/pmc_dec_8p2_w" "ecg_mm_kernel<8, 2" 5368709120 \
			"$O/pmc_traffic_dec_8p2.json" || exit $?
		python tools/pmc_traffic.py "$O/pmc_enc_16p2_f" "$O/pmc_enc_16p2_w" "ecg_mm_kernel<16, 2" 2415919104 \
			"$O/pmc_traffic_enc_16p2.json" || exit $?
		python tools/pmc_traffic.py "$O/pmc_dec_16p2_f" "$O/pmc_dec_16p2_w" "ecg_mm_kernel<16, 2" 2415919104 \
			"$O/pmc_traffic_dec_16p2.json" || exit $?
		;;
	updpmc)           # HBM bytes of the one-cell delta update kernel
		rm -rf "$O/pmc_upd_f" "$O/pmc_upd_w"
		step rocprof_upd_f 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv \
			-d "$O/pmc_upd_f" -o run -- python3 tools/ec_pmc.py upd1_8p2 || exit $?
		step rocprof_upd_w 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv \
			-d "$O/pmc_upd_w" -o run -- python3 tools/ec_pmc.py upd1_8p2 || exit $?
		python tools/pmc_traffic.py "$O/pmc_upd_f" "$O/pmc_upd_w" "ecg_mm_kernel<1, 2" 3221225472 \
			"$O/pmc_traffic_upd1_8p2.json" || exit $?
		;;
	ecdram)           # memory-side queueing of the EC shapes vs the streaming kernels: outstanding
	                  # requests per cycle (LEVEL), requests, DRAM-credit stall cycles, GRBM cycles
		for w in ${ECDRAM_SHAPES:-read write enc_4p2 enc_8p2 dec_8p2 enc_16p2 enc_16p2_cap2}; do
			rm -rf "$O/dram_${w}_r" "$O/dram_${w}_w"
			step dram_${w}_r 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ \
				TCC_EA0_RDREQ_LEVEL TCC_EA0_RDREQ_DRAM_CREDIT_STALL GRBM_GUI_ACTIVE --output-format csv \
				-d "$O/dram_${w}_r" -o run -- python3 tools/ec_pmc.py $w || exit $?
			step dram_${w}_w 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ \
				TCC_EA0_WRREQ_LEVEL TCC_EA0_WRREQ_DRAM_CREDIT_STALL GRBM_GUI_ACTIVE --output-format csv \
				-d "$O/dram_${w}_w" -o run -- python3 tools/ec_pmc.py $w || exit $?
			python tools/pmc_summary.py --skip 2 "$O/dram_${w}_r/run_counter_collection.csv" \
				"$O/dram_${w}_w/run_counter_collection.csv" > "$O/dram_${w}.jsonl" || exit $?
		done
		;;
	rehearse8)        # 8 ranks on this one GPU: rendezvous, NUMA pinning, legs, accounting (no scaling)
		step bench_rehearse8 900 python bench.py --gpus 8 --allow-shared-device --steps 10 --warmup 2 --no-cpu \
			|| exit $?
		;;
	dist2)            # 2 ranks through torch.distributed.run, one GPU shared
		step dist2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
			--master-port 29533 bench.py --gpus 2 --allow-shared-device --steps 5 --warmup 2 --no-cpu || exit $?
		;;
	hoststream)
		step hoststream_n1 300 python bench.py --workload rebuild_stream_8p2 --steps 5 --warmup 1 || exit $?
		;;
	ecab)             # EC_LIBS="name=path ...": product-kernel builds A/B (tools/ec_ab.py)
		step ec_ab 1000 python tools/ec_ab.py base=daos_amd/lib/libecg.so ${EC_LIBS:-} || exit $?
		;;
	exptests)         # EXP_LIBS="path ...": the product parity suites against each experimental build
		for lib in ${EXP_LIBS:-}; do
			tag=$(basename "$(dirname "$lib")")
			ECG_TEST_LIB=$lib step exptests_$tag 600 $PYTEST -x tests/test_gpu_parity.py tests/test_gpu_align.py \
				tests/test_gpu_configs.py tests/test_gpu_tuning.py
			rc=$?; [ $rc -eq 0 ] || exit $rc
		done
		;;
	unaligned)        # dword lanes at misaligned addresses vs the launch's own choice (tools/unaligned_ab.py)
		step unaligned_ab 300 python tools/unaligned_ab.py || exit $?
		;;
	csum)
		step bench_csum 600 python tools/bench_csum.py || exit $?
		;;
	crcsq)            # SQ / LDS counters of the standalone CRC kernels (tools/crc_pmc.py)
		rm -rf "$O/pmc_csq1"
		step rocprof_csq1 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT \
			SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU \
			SQ_ACTIVE_INST_LDS --output-format csv -d "$O/pmc_csq1" -o run -- python3 tools/crc_pmc.py standalone \
			|| exit $?
		;;
	pcie)
		step pcie 600 python tools/bench_pcie.py || exit $?
		;;
	dropin)
		step dropin_default 300 python tools/bench_dropin.py || exit $?
		DROPIN_DEVICE=1 step dropin_device 300 python tools/bench_dropin.py || exit $?
		for zc in 0 1048576; do
			ECG_DROPIN_CROSSOVER=0 ECG_ZERO_COPY_MAX=$zc step dropin_$zc 300 python tools/bench_dropin.py || exit $?
		done
		;;
	rebuild)
		step bench_rebuild 300 python tools/bench_rebuild.py || exit $?
		;;
	fillback)
		step bench_fillback 300 python tools/bench_fillback.py || exit $?
		;;
	sel)              # SEL="tests/x.py tests/y.py::t": a selection of the GPU suite
		step pytest_sel 900 $PYTEST -x -m gpu ${SEL:-tests/test_gpu_parity.py}
		rc=$?; [ $rc -le 1 ] || exit $rc
		;;
	dropinx)          # the drop-in crossover: CPU path vs GPU staging vs device cells (tools/dropin_bench.c)
		make -s -C tests/c dropin_bench > /dev/null || exit 2
		step dropin_bench 600 ./build/ctest/dropin_bench || exit $?
		;;
	qdev)             # device-cell drop-in calls and queue requests from T threads (tools/queue_bench.c device)
		make -s -C tests/c queue_bench > /dev/null || exit 2
		for C in 32768 131072 1048576; do
			for T in 1 2 4 8 16; do
				step qdev_${C}_$T 120 ./build/ctest/queue_bench $C $T device $((C > 131072 ? 128 : 1024)) || exit $?
			done
		done
		;;
	hsoverlap)        # configs[4]: serial vs overlapped host batches (tools/hoststream_overlap.py)
		step hoststream_overlap 300 python tools/hoststream_overlap.py || exit $?
		HS_TORCH=1 step hoststream_overlap_torch 300 python tools/hoststream_overlap.py || exit $?
		;;
	legprobe)         # configs[4] leg in phases (tools/leg_probe.py)
		step leg_probe 300 python tools/leg_probe.py || exit $?
		;;
	dthreads)         # host-cell drop-in calls from T threads, with and without a visible GPU
		make -s -C tests/c dropin_threads > /dev/null || exit 2
		for T in 1 8 16; do
			step dthreads_gpu_$T 120 ./build/ctest/dropin_threads 32768 $T || exit $?
			HIP_VISIBLE_DEVICES= step dthreads_nogpu_$T 120 ./build/ctest/dropin_threads 32768 $T || exit $?
			step dthreads_tiny_gpu_$T 120 ./build/ctest/dropin_threads 32768 $T 20000 8 tiny || exit $?
			HIP_VISIBLE_DEVICES= step dthreads_tiny_nogpu_$T 120 ./build/ctest/dropin_threads 32768 $T 20000 8 tiny || exit $?
		done
		;;
	dsoak)            # concurrent drop-in soak vs the oracle (tools/dropin_soak.py)
		step dropin_soak 600 python tools/dropin_soak.py || exit $?
		;;
	layoutab)         # parity-row placement x block order (tools/layout_ab.py)
		step layout_ab 600 python tools/layout_ab.py || exit $?
		;;
	qhost)            # host-cell one-stripe callers from T threads: drop-in (CPU path) / queue / oracle GFNI
		make -s -C tests/c queue_bench > /dev/null || exit 2
		for C in 32768 131072 1048576; do
			for T in 1 8 16; do
				step qhost_${C}_$T 120 ./build/ctest/queue_bench $C $T || exit $?
			done
		done
		;;
	ctest)
		make -C tests/c > /dev/null || exit 2
		step ctest 300 ./build/ctest/test_ecg_c || exit $?
		;;
	*)
		echo "unknown step $what"; exit 2
		;;
	esac
done
echo "== all done"

#!/bin/bash
# GPU-box driver for one gpurun call.  Every GPU step has its own time limit;
# any fault / abort / segfault / timeout ends the call (no retries).  Test
# failures (pytest exit 1) are not faults and do not stop later steps.
#   tools/gpu_run.sh [smoke] [tests] [bench] [prof] [pmc] [fulltests] [csumtests] [hoststream] [tune12] ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp

step() {   # name timeout cmd...
	local name=$1 to=$2
	shift 2
	echo "== $name: $*"
	timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
	local rc=$?
	echo "== $name rc=$rc"
	tail -n 12 "gpurun_out/$name.log"
	return $rc
}

for what in "$@"; do
	case $what in
	smoke)
		step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
		;;
	tests)
		step pytest_gpu 900 python -m pytest tests -q -m gpu -p no:cacheprovider -k "not full_size and not degraded_decode"
		rc=$?; [ $rc -le 1 ] || exit $rc
		;;
	fulltests)
		step pytest_gpu_full 900 python -m pytest tests -q -m gpu -p no:cacheprovider -k "full_size or degraded_decode"
		rc=$?; [ $rc -le 1 ] || exit $rc
		;;
	bench)
		step bench 900 python bench.py || exit $?
		;;
	prof)
		rm -rf gpurun_out/prof
		step rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
			-- python3 bench.py --steps 10 --warmup 2 --no-detail --no-cpu || exit $?
		;;
	pmc)
		rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
		step rocprof_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run \
			-- python3 bench.py --steps 4 --warmup 1 --no-detail --no-cpu --profile-only || exit $?
		step rocprof_write 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run \
			-- python3 bench.py --steps 4 --warmup 1 --no-detail --no-cpu --profile-only || exit $?
		;;
	tune)
		step tune 600 python tools/tune.py || exit $?
		;;
	tune2)
		step tune2 600 python tools/tune2.py || exit $?
		;;
	pcie)
		step pcie 600 python tools/bench_pcie.py || exit $?
		;;
	dist2)
		step dist2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
			--master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 || exit $?
		;;
	tune4)
		step tune4 600 python tools/tune4.py || exit $?
		;;
	tune5)
		step tune5 600 python tools/tune5.py || exit $?
		;;
	tune6)
		step tune6 600 python tools/tune6.py || exit $?
		;;
	tune7)
		step tune7 600 python tools/tune7.py || exit $?
		;;
	qbench)
		make -C tests/c > /dev/null || exit 2
		for c in 32768 131072 1048576; do
			for t in 8 16; do
				step qbench_${c}_$t 300 ./build/ctest/queue_bench $c $t || exit $?
			done
		done
		cat gpurun_out/qbench_*.log | grep '^{' > gpurun_out/qbench.jsonl
		;;
	qupdate)
		make -C tests/c > /dev/null || exit 2
		for c in 32768 131072 1048576; do
			step qupd_${c} 300 ./build/ctest/queue_bench $c 16 update || exit $?
		done
		cat gpurun_out/qupd_*.log | grep '^{' > gpurun_out/queue_update.jsonl
		;;
	ctest)
		make -C tests/c > /dev/null || exit 2
		step ctest 300 ./build/ctest/test_ecg_c || exit $?
		;;
	tune9)
		step tune9 600 python tools/tune9.py || exit $?
		;;
	tune8)
		step tune8 600 python tools/tune8.py || exit $?
		;;
	csum)
		step bench_csum 600 python tools/bench_csum.py || exit $?
		;;
	cpubase)
		step cpu_baselines 600 python tools/cpu_baselines.py || exit $?
		;;
	fillback)
		step bench_fillback 300 python tools/bench_fillback.py || exit $?
		;;
	fillback_prof)
		rm -rf gpurun_out/prof_fb
		step rocprof_fillback 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fb -o run \
			-- python3 tools/bench_fillback.py || exit $?
		;;
	dropin)
		rm -f gpurun_out/bench_dropin.jsonl
		for zc in 0 1048576 1073741824; do
			ECG_ZERO_COPY_MAX=$zc step dropin_$zc 300 python tools/bench_dropin.py || exit $?
		done
		;;
	rebuild)
		step bench_rebuild 300 python tools/bench_rebuild.py || exit $?
		;;
	tune10)
		step tune10 600 python tools/tune10.py || exit $?
		;;
	tune3)
		step tune3 600 python tools/tune3.py || exit $?
		;;
	tune12)
		step tune12 500 python tools/tune12.py || exit $?
		;;
	hoststream)
		step hoststream_n1 300 python bench.py --workload rebuild_stream_8p2 --steps 5 --warmup 1 || exit $?
		step hoststream_2rank 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
			--master-addr 127.0.0.1 --master-port 29541 bench.py --workload rebuild_stream_8p2 --gpus 2 \
			--steps 5 --warmup 1 || exit $?
		;;
	csumtests)
		step csum_tests 300 python -m pytest tests/test_gpu_csum.py tests/test_migrate.py tests/test_gpu_graph.py \
			-q -x -p no:cacheprovider
		rc=$?; [ $rc -eq 0 ] || exit $rc
		;;
	fusedcost)
		for lib in daos_amd/lib/libecg.so build/exp/libecg_NO_MULMOD.so build/exp/libecg_NO_CRC.so \
			   daos_amd/lib/libecg.so; do
			step fusedcost 300 python tools/fused_cost.py $lib || exit $?
			grep '^{' gpurun_out/fusedcost.log >> gpurun_out/fusedcost.jsonl
		done
		;;
	fusedstruct)
		for lib in build/exp/libecg_NONE.so daos_amd/lib/libecg.so; do
			FUSED_COST_COLS=1,2,4,8 step fusedcost 400 python tools/fused_cost.py $lib || exit $?
			grep '^{' gpurun_out/fusedcost.log >> gpurun_out/fusedcost.jsonl
		done
		;;
	tune13)
		step tune13 500 python tools/tune13.py || exit $?
		;;
	csumbench)
		step bench_csum 300 python tools/bench_csum.py || exit $?
		python - <<'PY'
import json
d = json.load(open("gpurun_out/bench_csum.json"))
for k, v in d.items():
    if k.startswith(("crc32", "shape_crc32", "enc_8p2")):
        print(k, v)
PY
		;;
	newtests)
		step pytest_new 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_multi.py -v -x \
			-p no:cacheprovider --timeout 300 --timeout-method thread
		rc=$?; [ $rc -le 1 ] || exit $rc
		;;
	alltests)
		step pytest_all 1000 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 \
			--timeout-method thread
		rc=$?; [ $rc -le 1 ] || exit $rc
		;;
	spawn2)
		step bench_spawn2 300 python bench.py --gpus 2 --allow-shared-device --steps 10 --warmup 2 \
			--no-detail --no-cpu || exit $?
		;;
	lib4)
		step bench_lib4 300 python bench.py --gpus 4 --sharder lib --allow-shared-device --steps 10 \
			--warmup 2 --no-detail || exit $?
		;;
	tune14)
		step tune14 600 python tools/tune14.py || exit $?
		;;
	tunetests)
		step pytest_tuning 300 python -u -m pytest tests/test_gpu_tuning.py -q -x -p no:cacheprovider \
			--timeout 120 --timeout-method thread
		rc=$?; [ $rc -le 1 ] || exit $rc
		;;
	crcpmc)
		rm -rf gpurun_out/pmc_lds
		step rocprof_lds 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
			--output-format csv -d gpurun_out/pmc_lds -o run -- python3 tools/crc_pmc.py fused || exit $?
		;;
	crcpmc2)
		rm -rf gpurun_out/pmc_sq1 gpurun_out/pmc_sq2
		step rocprof_sq1 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
			SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
			--output-format csv -d gpurun_out/pmc_sq1 -o run -- python3 tools/crc_pmc.py fused || exit $?
		step rocprof_sq2 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY \
			SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_WR \
			--output-format csv -d gpurun_out/pmc_sq2 -o run -- python3 tools/crc_pmc.py fused || exit $?
		;;
	crcsq)
		# standalone crc32 / crc64 kernels (32 KiB chunks, 1 GiB): SQ / LDS / GRBM counter passes
		rm -rf gpurun_out/pmc_csq1 gpurun_out/pmc_csq2 gpurun_out/pmc_cgrbm
		step rocprof_csq1 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES \
			SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY \
			--output-format csv -d gpurun_out/pmc_csq1 -o run -- python3 tools/crc_pmc.py || exit $?
		step rocprof_csq2 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS \
			SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
			--output-format csv -d gpurun_out/pmc_csq2 -o run -- python3 tools/crc_pmc.py || exit $?
		step rocprof_cgrbm 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT \
			--output-format csv -d gpurun_out/pmc_cgrbm -o run -- python3 tools/crc_pmc.py || exit $?
		python tools/pmc_summary.py --skip 1 gpurun_out/pmc_csq1/run_counter_collection.csv \
			gpurun_out/pmc_csq2/run_counter_collection.csv gpurun_out/pmc_cgrbm/run_counter_collection.csv \
			> gpurun_out/crc_sq_summary.jsonl || exit $?
		;;
	fusedab)
		step fused_tables_ab 600 python tools/fused_tables_ab.py 8,2,512 4,2,1024 16,2,256 8,1,512 || exit $?
		;;
	hostlib)
		step hoststream_lib2 300 python bench.py --workload rebuild_stream_8p2 --gpus 2 --sharder lib \
			--allow-shared-device --steps 5 --warmup 1 || exit $?
		step hoststream_n1 300 python bench.py --workload rebuild_stream_8p2 --steps 5 --warmup 1 || exit $?
		;;
	fusedblocked)
		step fused_blocked 600 python tools/fused_blocked.py || exit $?
		;;
	fusedcols)
		step fused_cols_ab 600 python tools/fused_cols_ab.py || exit $?
		;;
	placement)
		step placement_sweep 600 python tools/placement_sweep.py || exit $?
		;;
	placealloc)
		step placement_alloc 600 python tools/placement_alloc.py || exit $?
		;;
	pmcjson)
		python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write "ecg_mm_kernel<4, 2" 6442450944 \
			gpurun_out/pmc_traffic.json || exit $?
		;;
	crcab)
		step crc_ab 600 python tools/crc_ab.py || exit $?
		;;
	eclibs)
		step ec_libs 900 python tools/ec_libs.py daos_amd/lib/libecg.so ${EC_LIBS:-build/exp/xoronly/libecg.so} || exit $?
		;;
	fusedlibs)
		step fused_libs 900 python tools/fused_libs.py daos_amd/lib/libecg.so ${FUSED_LIBS:-} || exit $?
		;;
	crclibs)
		step crc_libs 900 python tools/crc_libs.py daos_amd/lib/libecg.so ${CRC_LIBS:-} || exit $?
		;;
	fusedpmc)
		rm -rf gpurun_out/pmc_ffetch gpurun_out/pmc_fwrite
		step rocprof_ffetch 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv \
			-d gpurun_out/pmc_ffetch -o run -- python3 tools/crc_pmc.py fused || exit $?
		step rocprof_fwrite 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv \
			-d gpurun_out/pmc_fwrite -o run -- python3 tools/crc_pmc.py fused || exit $?
		;;
	fusedsq)
		# FUSED_LIB=path: counters of an experimental build instead (e.g. -DECG_EXP_NO_CRC)
		lib=${FUSED_LIB:+--lib=$FUSED_LIB}
		tag=${FUSED_TAG:-}
		rm -rf gpurun_out/pmc_fsq1$tag gpurun_out/pmc_fsq2$tag gpurun_out/pmc_fgrbm$tag
		step rocprof_fsq1$tag 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES \
			SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY \
			--output-format csv -d gpurun_out/pmc_fsq1$tag -o run -- python3 tools/fused_pmc.py $lib || exit $?
		step rocprof_fsq2$tag 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS \
			SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
			--output-format csv -d gpurun_out/pmc_fsq2$tag -o run -- python3 tools/fused_pmc.py $lib || exit $?
		step rocprof_fgrbm$tag 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT \
			--output-format csv -d gpurun_out/pmc_fgrbm$tag -o run -- python3 tools/fused_pmc.py $lib || exit $?
		python tools/pmc_summary.py --skip 6 gpurun_out/pmc_fsq1$tag/run_counter_collection.csv \
			gpurun_out/pmc_fsq2$tag/run_counter_collection.csv gpurun_out/pmc_fgrbm$tag/run_counter_collection.csv \
			> gpurun_out/fused_sq_summary$tag.jsonl || exit $?
		;;
	ecpmc)
		for w in dec_8p2 enc_16p2 dec_16p2; do
			rm -rf gpurun_out/pmc_${w}_f gpurun_out/pmc_${w}_w
			step rocprof_${w}_f 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv \
				-d gpurun_out/pmc_${w}_f -o run -- python3 tools/ec_pmc.py $w || exit $?
			step rocprof_${w}_w 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv \
				-d gpurun_out/pmc_${w}_w -o run -- python3 tools/ec_pmc.py $w || exit $?
		done
		python tools/pmc_traffic.py gpurun_out/pmc_dec_8p2_f gpurun_out/pmc_dec_8p2_w "ecg_mm_kernel<8, 2" \
			5368709120 gpurun_out/pmc_traffic_dec_8p2.json || exit $?
		python tools/pmc_traffic.py gpurun_out/pmc_enc_16p2_f gpurun_out/pmc_enc_16p2_w "ecg_mm_kernel<16, 2" \
			2415919104 gpurun_out/pmc_traffic_enc_16p2.json || exit $?
		python tools/pmc_traffic.py gpurun_out/pmc_dec_16p2_f gpurun_out/pmc_dec_16p2_w "ecg_mm_kernel<16, 2" \
			2415919104 gpurun_out/pmc_traffic_dec_16p2.json || exit $?
		;;
	exp)
		# EXP_LIBS="build/exp/a/libecg.so ...": checksum parity of each experimental build, then the fused A/B
		for lib in ${EXP_LIBS}; do
			tag=$(basename "$(dirname "$lib")")
			ECG_TEST_LIB=$lib step exptests_$tag 300 python -u -m pytest tests/test_gpu_csum.py tests/test_migrate.py \
				-q -x -p no:cacheprovider --timeout 120 --timeout-method thread
			rc=$?; [ $rc -eq 0 ] || exit $rc
		done
		FUSED_ROUNDS=${FUSED_ROUNDS:-3} step fused_libs 900 python tools/fused_libs.py daos_amd/lib/libecg.so ${EXP_LIBS} \
			|| exit $?
		;;
	dist4)
		step dist4 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
			--master-port 29537 bench.py --gpus 4 --steps 20 --warmup 3 || exit $?
		;;
	*)
		echo "unknown step $what"; exit 2
		;;
	esac
done
echo "== all done"

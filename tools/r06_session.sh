#!/usr/bin/env bash
# Round-6 GPU session: tools/r06_session.sh STEP...
# Each step has its own time limit; a failure other than test failures stops the session.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {   # step NAME TIMEOUT CMD...
    local name=$1 to=$2; shift 2
    echo "== $name (timeout ${to}s) =="
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    tail -n 5 "$OUT/$name.log"
    echo "== $name rc=$rc =="
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
    return 0
}
PYT="python -u -m pytest -x -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider"
for s in "$@"; do
    case $s in
        new) step pytest_new 500 $PYT tests/test_multi_device.py tests/test_dropin.py -m gpu ;;
        spec) step pytest_spec 300 $PYT tests/test_speculation.py -m gpu ;;
        gridres)   # candidate-table resolution: superset sizes per build, then khaslana A/B
            for v in ${GRID_VARS:-s16b16 s24b24}; do
                PTAMD_LIB=$PWD/project3-cuda-path-tracer-2025_amd/build/ab/$v.so PT_SECTIONS_SKIP_CAMERA=1 \
                    step sec_kh_$v 300 python -u tools/section_times.py --scene cornell_obj_khaslana --res 1600x1600 --depth 12 --variant 190 --frames 8 --out gpurun_out/sec_kh_$v.json
            done
            PT_SECTIONS_SKIP_CAMERA=1 step sec_kh_base 300 python -u tools/section_times.py --scene cornell_obj_khaslana --res 1600x1600 --depth 12 --variant 190 --frames 8 --out gpurun_out/sec_kh_base.json
            L=project3-cuda-path-tracer-2025_amd/build
            AB_ROUNDS=2 AB_LIBS="$L/libptamd.so ${GRID_AB:-$L/ab/g16b16.so $L/ab/s16b16.so $L/ab/s16b32.so $L/ab/s24b24.so}" AB_TAG=gridres_khaslana \
                AB_ARGS="--steps 32 --warmup 2 --scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12" step ab_gridres_khaslana 900 bash tools/ab_libs.sh ;;
        gridab)   # the old 8 / 8 full table (build/ab/old.so) against the product build
            L=project3-cuda-path-tracer-2025_amd/build
            for sc in ${GRID_SCENES:-cornell_obj_khaslana cornell_obj_cyrene cornell_obj_phainon}; do
                X=""; [ $sc = cornell_obj_khaslana ] && X="--res 1600x1600 --depth 12"
                AB_ROUNDS=3 AB_LIBS="$L/ab/${GRID_OLD:-old}.so $L/libptamd.so" AB_TAG=grid_$sc \
                    AB_ARGS="--steps 24 --warmup 2 --scene scenes/$sc.json $X" step ab_grid_$sc 600 bash tools/ab_libs.sh
            done ;;
        khprof)   # khaslana's kernel stats, PMC traffic and sections at the current build
            rm -rf gpurun_out/prof_c5_khaslana gpurun_out/pmc/khtr_p*
            step prof_c5_khaslana 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_khaslana -o run --output-format csv -- python bench.py --no-cpu-baseline --no-configs --no-api --no-spread --steps 32 --warmup 2 --scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12
            PMC_TAG=khtr_ PMC_STEPS=8 PMC_WARMUP=2 PMC_SETS="FETCH_SIZE;WRITE_SIZE" step pmc_khtr 400 bash tools/pmc.sh --scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12
            PT_SECTIONS_SKIP_CAMERA=1 step sec_khaslana 300 python -u tools/section_times.py --scene cornell_obj_khaslana --res 1600x1600 --depth 12 --variant 190 --frames 8 --out gpurun_out/sec_khaslana.json ;;
        cyrprof)   # the 262k stand-in's kernel stats, PMC traffic and sections at the current build
            rm -rf gpurun_out/prof_m262k_cyrene gpurun_out/pmc/cyr_p*
            step prof_m262k_cyrene 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_m262k_cyrene -o run --output-format csv -- python bench.py --no-cpu-baseline --no-configs --no-api --no-spread --steps 24 --warmup 2 --scene scenes/cornell_obj_cyrene.json
            PMC_TAG=cyr_ PMC_STEPS=16 PMC_WARMUP=2 PMC_SETS="FETCH_SIZE;WRITE_SIZE" step pmc_cyr 400 bash tools/pmc.sh --scene scenes/cornell_obj_cyrene.json
            step sec_cyrene 300 python -u tools/section_times.py --scene cornell_obj_cyrene --variant 190 --frames 16 --out gpurun_out/sec_cyrene.json ;;
        cfgpmc)   # PMC traffic of the sub-records that had none (bench.py traffic_file names)
            T="FETCH_SIZE;WRITE_SIZE"
            PMC_TAG=c2g_ PMC_SETS="$T" step pmc_c2g 300 bash tools/pmc.sh --scene scenes/cornell_glass_test.json --sort
            PMC_TAG=c2o_ PMC_SETS="$T" step pmc_c2o 300 bash tools/pmc.sh --scene scenes/cornell_glass_test.json
            PMC_TAG=phn_ PMC_STEPS=16 PMC_WARMUP=2 PMC_SETS="$T" step pmc_phn 400 bash tools/pmc.sh --scene scenes/cornell_obj_phainon.json
            PMC_TAG=cyrn_ PMC_STEPS=8 PMC_WARMUP=1 PMC_SETS="$T" step pmc_cyrn 400 bash tools/pmc.sh --scene scenes/cornell_obj_cyrene.json --variant 250
            PMC_TAG=phnn_ PMC_STEPS=8 PMC_WARMUP=1 PMC_SETS="$T" step pmc_phnn 400 bash tools/pmc.sh --scene scenes/cornell_obj_phainon.json --variant 250 ;;
        khvar)   # khaslana traffic with a variant library (KH_LIB), then the A/B against the product
            PTAMD_LIB=$PWD/$KH_LIB PMC_TAG=khv_ PMC_STEPS=8 PMC_WARMUP=2 PMC_SETS="FETCH_SIZE;WRITE_SIZE" step pmc_khv 400 bash tools/pmc.sh --scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12
            L=project3-cuda-path-tracer-2025_amd/build
            AB_ROUNDS=3 AB_LIBS="$L/libptamd.so $KH_LIB" AB_TAG=khvar \
                AB_ARGS="--steps 32 --warmup 2 --scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12" step ab_khvar 600 bash tools/ab_libs.sh ;;
        phnpmc) rm -rf gpurun_out/pmc/phn_p*
            PMC_TAG=phn_ PMC_STEPS=16 PMC_WARMUP=2 PMC_SETS="FETCH_SIZE;WRITE_SIZE" step pmc_phn 400 bash tools/pmc.sh --scene scenes/cornell_obj_phainon.json ;;
        glibc) step pytest_glibc 300 $PYT tests/test_gpu_parity.py -m gpu -k statistical ;;
        meshlib) PTAMD_LIB=$PWD/${MESH_LIB} step pytest_meshlib 600 $PYT tests/test_gpu_parity.py tests/test_ref_pins.py tests/test_speculation.py -m gpu -k "bnnuy or khaslana or bvh or mesh or candidate or config5 or intersections or speculated" ;;
        mesh) step pytest_mesh 600 $PYT tests/test_gpu_parity.py tests/test_ref_pins.py -m gpu -k "bnnuy or khaslana or bvh or mesh or candidate or config5 or intersections" ;;
        gpu) step pytest_gpu 900 $PYT tests -m gpu ;;
        smoke) step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) step bench_k20 400 python bench.py --steps 20 --warmup 5 ;;
        benchq) step bench_q 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-api --no-spread ;;
        calib) step calib_plain 120 project3-cuda-path-tracer-2025_amd/build/fetch_calib
            step calib_pmc 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/calib -o run --output-format csv -- project3-cuda-path-tracer-2025_amd/build/fetch_calib
            step calib_pmc_hit 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/calib_hit -o run --output-format csv -- project3-cuda-path-tracer-2025_amd/build/fetch_calib ;;
        calibreq) step calib_req 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d gpurun_out/calib_req -o run --output-format csv -- project3-cuda-path-tracer-2025_amd/build/fetch_calib
            step calib_bubble 120 rocprofv3 --kernel-trace --pmc TCC_BUBBLE_sum WRITE_SIZE -d gpurun_out/calib_bubble -o run --output-format csv -- project3-cuda-path-tracer-2025_amd/build/fetch_calib ;;
        meshreq) R="TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_32B_sum,TCC_EA0_RDREQ_64B_sum,TCC_EA0_RDREQ_128B_sum"
            PMC_TAG=req_fused_ PMC_SETS="$R" step pmc_req_fused 300 bash tools/pmc.sh
            PMC_TAG=req_bunny_ PMC_SETS="$R" step pmc_req_bunny 300 bash tools/pmc.sh --scene scenes/cornell_obj_bnnuy.json
            PMC_TAG=req_kh_ PMC_STEPS=8 PMC_WARMUP=2 PMC_SETS="$R" step pmc_req_kh 300 bash tools/pmc.sh --scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12
            PMC_TAG=req_cyr_ PMC_STEPS=16 PMC_WARMUP=2 PMC_SETS="$R" step pmc_req_cyr 300 bash tools/pmc.sh --scene scenes/cornell_obj_cyrene.json ;;
        cyrhit) PMC_TAG=cyrhit_ PMC_STEPS=16 PMC_WARMUP=2 PMC_SETS="TCC_HIT_sum,TCC_MISS_sum" step pmc_cyr_hit 300 bash tools/pmc.sh --scene scenes/cornell_obj_cyrene.json
            PMC_TAG=bunhit_ PMC_SETS="TCC_HIT_sum,TCC_MISS_sum" step pmc_bunny_hit 300 bash tools/pmc.sh --scene scenes/cornell_obj_bnnuy.json ;;
        bandprobe) step band_probe 200 python tools/band_copy_probe.py ;;
        multi) step multi_probe 300 python tools/multi_probe.py 20 ;;
        multidirect) PT_MULTI_F1_DIRECT=1 step multi_probe_direct 300 python tools/multi_probe.py 20 ;;
        inproc) step inproc 200 python bench.py --gpus 2 --inproc --inproc-devices 0,0 --steps 20 --warmup 5 ;;
        ab_*)   # ab_<tag>: AB_LIBS / AB_ROUNDS from the environment, scenes below
            tag=${s#ab_}
            B=project3-cuda-path-tracer-2025_amd/build/ab
            [ -z "${AB_SKIP_CORNELL:-}" ] && AB_TAG=${tag}_cornell AB_ARGS="--steps 20 --warmup 5" step ab_${tag}_cornell 400 bash tools/ab_libs.sh
            AB_TAG=${tag}_bunny AB_ARGS="--steps 20 --warmup 5 --scene scenes/cornell_obj_bnnuy.json" step ab_${tag}_bunny 500 bash tools/ab_libs.sh
            AB_TAG=${tag}_khaslana AB_ARGS="--steps 10 --warmup 2 --scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12" step ab_${tag}_khaslana 600 bash tools/ab_libs.sh ;;
        profiles) step profiles 1100 bash tools/r06_profiles.sh ;;
        profstats) step profiles_stats 600 bash tools/r06_profiles.sh stats ;;
        profpmc) step profiles_pmc 900 bash tools/r06_profiles.sh pmc ;;
        profsec) step profiles_sec 600 bash tools/r06_profiles.sh sections ;;
        apicopy)
            step prof_api_copy 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_api_copy -o run --output-format csv -- python tools/api_trace.py run copy
            python tools/api_trace.py overlap gpurun_out/prof_api_copy/run_kernel_trace.csv gpurun_out/prof_api_copy/run_memory_copy_trace.csv --out gpurun_out/api_copy_overlap.json ;;
        benchapi) step bench_api 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-configs --no-spread ;;
        hist) step sec_bunny 300 python -u tools/section_times.py --scene cornell_obj_bnnuy --variant 190 --frames 16 --out gpurun_out/sec_bunny.json
            step sec_khaslana 300 python -u tools/section_times.py --scene cornell_obj_khaslana --res 1600x1600 --depth 12 --variant 190 --frames 8 --out gpurun_out/sec_khaslana.json ;;
        large) step pytest_large 600 $PYT tests/test_large_mesh.py -m gpu ;;
        multitest) step pytest_multi 600 $PYT tests/test_multi_device.py tests/test_speculation.py tests/test_dropin.py -m gpu ;;
        benchlarge) B="python bench.py --no-cpu-baseline --no-configs --no-api --no-spread"
            step bench_cyrene 300 $B --steps 24 --warmup 2 --scene scenes/cornell_obj_cyrene.json
            step bench_cyrene_nodes 300 $B --steps 8 --warmup 1 --scene scenes/cornell_obj_cyrene.json --variant 250
            step bench_phainon 300 $B --steps 24 --warmup 2 --scene scenes/cornell_obj_phainon.json
            step bench_phainon_nodes 300 $B --steps 8 --warmup 1 --scene scenes/cornell_obj_phainon.json --variant 250 ;;
        tailtest) step pytest_tail 400 $PYT tests/test_bvh_tail.py -m gpu ;;
        meshlanes) PT_BVH_TAIL_LANES=${MESH_TAIL:-16} step pytest_meshlanes 600 $PYT tests/test_gpu_parity.py tests/test_speculation.py -m gpu -k "bnnuy or khaslana or bvh or mesh or config5 or speculated" ;;
        laneab) ARMS="${LANE_ARMS:-PT_BVH_TAIL_LANES=0 PT_BVH_TAIL_LANES=16 PT_BVH_TAIL_LANES=24 PT_BVH_TAIL_LANES=32}"
            AB_TAG=lane_bunny AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_bnnuy.json" step ab_lane_bunny 900 bash tools/ab_env.sh
            AB_TAG=lane_khaslana AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12" step ab_lane_khaslana 900 bash tools/ab_env.sh ;;
        meshstats) B="python bench.py --no-cpu-baseline --no-configs --no-api --no-spread"
            step prof_c4_bunny 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4_bunny -o run --output-format csv -- $B --steps 48 --warmup 4 --scene scenes/cornell_obj_bnnuy.json
            step prof_c5_khaslana 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_khaslana -o run --output-format csv -- $B --steps 32 --warmup 2 --scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12 ;;
        occab) ARMS="- PT_BVH_LDS_PAD=5120 PT_BVH_LDS_PAD=11264"
            AB_ROUNDS=2 AB_TAG=occ_bunny AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_bnnuy.json" step ab_occ_bunny 900 bash tools/ab_env.sh ;;
        qorderab) ARMS="${ORDER_ARMS:-- PT_BVH_BFS_LEVELS=0 PT_BVH_BFS_LEVELS=8 PT_BVH_BFS_LEVELS=18}"
            AB_ROUNDS=2 AB_TAG=qorder_cyrene AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_cyrene.json --steps 24 --warmup 2" step ab_qorder_cyrene 900 bash tools/ab_env.sh
            AB_ROUNDS=2 AB_TAG=qorder_phainon AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_phainon.json --steps 24 --warmup 2" step ab_qorder_phainon 900 bash tools/ab_env.sh ;;
        tailtune) ARMS="${TAIL_ARMS:-- PT_BVH_TAIL_REFILL=8 PT_BVH_TAIL_REFILL=32 PT_BVH_TAIL_TRAV_BLOCKS=160 PT_BVH_TAIL_TRAV_BLOCKS=320}"
            AB_ROUNDS=2 AB_TAG=tailtune_cyrene AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_cyrene.json --steps 24 --warmup 2" step ab_tailtune_cyrene 900 bash tools/ab_env.sh
            AB_ROUNDS=2 AB_TAG=tailtune_bunny AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_bnnuy.json" step ab_tailtune_bunny 900 bash tools/ab_env.sh ;;
        spilltest) step pytest_spill 600 $PYT tests/test_large_mesh.py -m gpu -k "spilled or four_wide" ;;
        spillab) ARMS="${SPILL_ARMS:-- PT_BVH_STACK_LDS=22 PT_BVH_STACK_LDS=16}"
            AB_ROUNDS=2 AB_TAG=spill_cyrene AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_cyrene.json --steps 24 --warmup 2" step ab_spill_cyrene 900 bash tools/ab_env.sh
            AB_ROUNDS=2 AB_TAG=spill_khaslana AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12 --steps 32 --warmup 2" step ab_spill_khaslana 900 bash tools/ab_env.sh
            AB_ROUNDS=2 AB_TAG=spill_bunny AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_bnnuy.json" step ab_spill_bunny 900 bash tools/ab_env.sh
            AB_ROUNDS=2 AB_TAG=spill_phainon AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_phainon.json --steps 24 --warmup 2" step ab_spill_phainon 900 bash tools/ab_env.sh ;;
        treeinfo) step tree_info 300 python -u tools/tree_info.py ;;
        quadlanes) ARMS="${LANE_ARMS:-PT_BVH_TAIL_LANES=32 PT_BVH_TAIL_LANES=40 PT_BVH_TAIL_LANES=48 PT_BVH_TAIL_LANES=56}"
            AB_ROUNDS=2 AB_TAG=qlanes_bunny AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_bnnuy.json" step ab_qlanes_bunny 900 bash tools/ab_env.sh
            AB_ROUNDS=2 AB_TAG=qlanes_khaslana AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12 --steps 32 --warmup 2" step ab_qlanes_khaslana 900 bash tools/ab_env.sh
            AB_ROUNDS=2 AB_TAG=qlanes_cyrene AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_cyrene.json --steps 24 --warmup 2" step ab_qlanes_cyrene 900 bash tools/ab_env.sh ;;
        quadtest) step pytest_quad 600 $PYT tests/test_large_mesh.py -m gpu -k "four_wide" ;;
        quadab) ARMS="${QUAD_ARMS:-PT_BVH_QUAD=0 PT_BVH_QUAD=1}"
            AB_ROUNDS=3 AB_TAG=quad_cyrene AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_cyrene.json --steps 24 --warmup 2" step ab_quad_cyrene 900 bash tools/ab_env.sh
            AB_ROUNDS=2 AB_TAG=quad_phainon AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_phainon.json --steps 24 --warmup 2" step ab_quad_phainon 900 bash tools/ab_env.sh
            AB_ROUNDS=2 AB_TAG=quad_bunny AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_bnnuy.json" step ab_quad_bunny 900 bash tools/ab_env.sh
            AB_ROUNDS=2 AB_TAG=quad_khaslana AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12 --steps 32 --warmup 2" step ab_quad_khaslana 900 bash tools/ab_env.sh ;;
        tpab) L=$PWD/project3-cuda-path-tracer-2025_amd/build/ab
            ARMS="PTAMD_LIB=$L/tp0.so -"
            AB_ROUNDS=3 AB_TAG=tp_bunny AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_bnnuy.json" step ab_tp_bunny 900 bash tools/ab_env.sh
            AB_ROUNDS=3 AB_TAG=tp_khaslana AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12 --steps 32 --warmup 2" step ab_tp_khaslana 900 bash tools/ab_env.sh
            AB_ROUNDS=3 AB_TAG=tp_cyrene AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_cyrene.json --steps 24 --warmup 2" step ab_tp_cyrene 900 bash tools/ab_env.sh ;;
        tptraffic) PMC_TAG=tpbun_ PMC_SETS="FETCH_SIZE;WRITE_SIZE" step pmc_tp_bunny 300 bash tools/pmc.sh --scene scenes/cornell_obj_bnnuy.json
            PMTAG=x PTAMD_LIB=$PWD/project3-cuda-path-tracer-2025_amd/build/ab/tp0.so PMC_TAG=tp0bun_ PMC_SETS="FETCH_SIZE;WRITE_SIZE" step pmc_tp0_bunny 300 bash tools/pmc.sh --scene scenes/cornell_obj_bnnuy.json ;;
        cyrmix) IM="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_BRANCH,SQ_INSTS_SMEM,SQ_INSTS_VMEM,SQ_WAVE_CYCLES;SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_WAIT_INST_ANY,GRBM_GUI_ACTIVE,TA_BUSY_avr,TA_TA_BUSY_sum"
            PMC_TAG=imcyr_ PMC_STEPS=16 PMC_WARMUP=2 PMC_SETS="$IM" step pmc_mix_cyr 300 bash tools/pmc.sh --scene scenes/cornell_obj_cyrene.json
            PMC_TAG=imbun_ PMC_SETS="$IM" step pmc_mix_bunny 300 bash tools/pmc.sh --scene scenes/cornell_obj_bnnuy.json ;;
        heightab) ARMS="${HEIGHT_ARMS:-PT_BVH_MAX_HEIGHT=0 - PT_BVH_MAX_HEIGHT=19}"
            AB_ROUNDS=2 AB_TAG=height_cyrene AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_cyrene.json --steps 24 --warmup 2" step ab_height_cyrene 900 bash tools/ab_env.sh
            AB_ROUNDS=2 AB_TAG=height_phainon AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_phainon.json --steps 24 --warmup 2" step ab_height_phainon 900 bash tools/ab_env.sh
            AB_ROUNDS=2 AB_TAG=height_khaslana AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12 --steps 32 --warmup 2" step ab_height_khaslana 900 bash tools/ab_env.sh ;;
        orderab) ARMS="${ORDER_ARMS:-- PT_BVH_BFS_LEVELS=0 PT_BVH_BFS_LEVELS=8 PT_BVH_BFS_LEVELS=12}"
            AB_ROUNDS=2 AB_TAG=order_cyrene AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_cyrene.json --steps 24 --warmup 2" step ab_order_cyrene 900 bash tools/ab_env.sh
            AB_ROUNDS=2 AB_TAG=order_phainon AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_phainon.json --steps 24 --warmup 2" step ab_order_phainon 900 bash tools/ab_env.sh
            AB_ROUNDS=2 AB_TAG=order_bunny AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_bnnuy.json" step ab_order_bunny 900 bash tools/ab_env.sh ;;
        lanesall) ARMS="${LANE_ARMS:-PT_BVH_TAIL_LANES=32 PT_BVH_TAIL_LANES=40 PT_BVH_TAIL_LANES=48 PT_BVH_TAIL_LANES=56}"
            AB_ROUNDS=2 AB_TAG=lanes_bunny AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_bnnuy.json" step ab_lanes_bunny 900 bash tools/ab_env.sh
            AB_ROUNDS=2 AB_TAG=lanes_khaslana AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12 --steps 32 --warmup 2" step ab_lanes_khaslana 900 bash tools/ab_env.sh
            AB_ROUNDS=2 AB_TAG=lanes_cyrene2 AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_cyrene.json --steps 24 --warmup 2" step ab_lanes_cyrene2 900 bash tools/ab_env.sh ;;
        lanesbig) ARMS="${LANE_ARMS:-PT_BVH_TAIL_LANES=0 PT_BVH_TAIL_LANES=16 PT_BVH_TAIL_LANES=32 PT_BVH_TAIL_LANES=48}"
            AB_ROUNDS=2 AB_TAG=lanes_cyrene AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_cyrene.json --steps 24 --warmup 2" step ab_lanes_cyrene 900 bash tools/ab_env.sh
            AB_ROUNDS=2 AB_TAG=lanes_phainon AB_ENVS="$ARMS" AB_ARGS="--scene scenes/cornell_obj_phainon.json --steps 24 --warmup 2" step ab_lanes_phainon 900 bash tools/ab_env.sh ;;
        empty) step empty_probe 120 project3-cuda-path-tracer-2025_amd/build/empty_block_probe ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo "session done"

#!/bin/bash
# Guarded GPU session for gpurun: every GPU step has its own time limit; the
# script stops at the first step that faults, aborts or times out (statuses
# other than 0 and pytest's 1 = "tests failed").
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIB=sac-gat-her_transportationrl_amd/trafficrl/libtrafficrl.so
sha256sum $LIB | cut -c1-16 > gpurun_out/lib_sha16.txt
step() {  # step <name> <timeout-seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 25 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
    return 0
}
# four rocprofv3 --pmc passes (each within gfx950's per-pass slots: 8 SQ, 4 TCC, 2 GRBM)
PMC_SETS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
          "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
          "FETCH_SIZE" "WRITE_SIZE")
pmc4() {  # pmc4 <name> <cmd...>: passes gpurun_out/<name>_p1..p4
    local name=$1; shift
    local k=1
    for set in "${PMC_SETS[@]}"; do
        step ${name}_p$k 300 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/${name}_p$k -o run --output-format csv -- "$@" || return 1
        k=$((k + 1))
    done
}
for s in "$@"; do
    case $s in
        tests) step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
        testsall) step gpu_tests 900 python -m pytest tests -m gpu -q ;;
        smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) step bench 600 python bench.py ;;
        benchq) step bench 400 python bench.py --steps 44 --warmup 22 --cpu-seconds 5 ;;
        benchenv) step bench_env 400 python bench.py --workload env --steps 66 --warmup 22 --no-cpu ;;
        benchtorch) step bench_torch 400 python bench.py --sp torch --steps 44 --warmup 22 --no-cpu
                    step bench_env_torch 400 python bench.py --workload env --sp torch --steps 66 --warmup 22 --no-cpu ;;
        benchgreedy) step bench_greedy 400 python bench.py --workload greedy --iters 60 --cpu-seconds 5 &&
                     step bench_greedy30 400 python bench.py --workload greedy --iters 30 --cpu-seconds 5 ;;
        benchfw) step bench_fw 400 python bench.py --method fw --steps 44 --warmup 22 --cpu-seconds 5 ;;
        benchana) step bench_ana 600 python bench.py --network anaheim --steps 10 --warmup 3 --cpu-seconds 5 ;;
        benchrand) step bench_rand 400 python bench.py --workload env --damage random --steps 66 --warmup 22 --no-cpu ;;
        envtests) step env_tests 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sparse.py tests/test_gpu_fallback.py tests/test_torch_sp.py tests/test_rewards.py tests/test_replay_train.py -m gpu -x -v --timeout 120 --timeout-method thread ;;
        obstests) step obs_tests 400 python -u -m pytest tests/test_gpu_parity.py tests/test_oracle_observe.py tests/test_gpu_gp.py tests/test_rewards.py tests/test_torch_sp.py -m gpu -x -q --timeout 120 --timeout-method thread ;;
        largetests) step large_tests 400 python -u -m pytest tests/test_gpu_large.py -m gpu -x -q --timeout 300 --timeout-method thread ;;
        profana) step profana 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profana -o run --output-format csv -- python3 bench.py --network anaheim --steps 6 --warmup 2 --no-cpu ;;
        pertests) step per_tests 300 python -u -m pytest tests/test_per_tree.py tests/test_replay_train.py -x -v --timeout 120 --timeout-method thread ;;
        prof) step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 44 --warmup 22 --no-cpu ;;
        profenv) step profenv 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profenv -o run --output-format csv -- python3 bench.py --workload env --steps 44 --warmup 22 --no-cpu ;;
        pmc) step pmc1 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d gpurun_out/pmc1 -o run --output-format csv -- python3 bench.py --workload env --steps 22 --warmup 0 --no-cpu
             step pmc2 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc2 -o run --output-format csv -- python3 bench.py --workload env --steps 22 --warmup 0 --no-cpu
             step pmc3 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc3 -o run --output-format csv -- python3 bench.py --workload env --steps 22 --warmup 0 --no-cpu
             step pmc4 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc4 -o run --output-format csv -- python3 bench.py --workload env --steps 22 --warmup 0 --no-cpu ;;
        profrand) step profrand 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profrand -o run --output-format csv -- python3 bench.py --workload env --damage random --steps 44 --warmup 22 --no-cpu ;;
        # raw counter CSVs stay on the box (gpurun copies back <= 64 MiB): summarised there
        # into profiles/r06_<name>_pmc.json (tools/pmc_summary.py, same library)
        pmcenv) pmc4 pmcenv python3 bench.py --workload env --steps 22 --warmup 0 --no-cpu &&
                python tools/pmc_summary.py r06_sf "pmcenv_p*" env_kernel > gpurun_out/pmcenv_summary.log 2>&1
                cp profiles/r06_sf_pmc.json gpurun_out/; rm -rf gpurun_out/pmcenv_p* ;;
        pmcana) pmc4 pmcana python3 bench.py --network anaheim --steps 6 --warmup 2 --no-cpu &&
                python tools/pmc_summary.py r06_ana "pmcana_p*" env_kernel_big > gpurun_out/pmcana_summary.log 2>&1
                cp profiles/r06_ana_pmc.json gpurun_out/; rm -rf gpurun_out/pmcana_p* ;;
        pmcact) pmc4 pmcact python3 tools/agent_profile.py 4096 act &&
                python tools/pmc_summary.py r06_act "pmcact_p*" gat_layer gat_mid edge_head gat_prologue Cijk > gpurun_out/pmcact_summary.log 2>&1
                cp profiles/r06_act_pmc.json gpurun_out/; rm -rf gpurun_out/pmcact_p* ;;
        pmcupd) pmc4 pmcupd python3 tools/agent_profile.py 4096 update &&
                python tools/pmc_summary.py r06_upd "pmcupd_p*" trx:: Cijk > gpurun_out/pmcupd_summary.log 2>&1
                cp profiles/r06_upd_pmc.json gpurun_out/; rm -rf gpurun_out/pmcupd_p* ;;
        stamps) step stamps 300 python tools/phase_stamps.py 4096 ;;
        stampsrand)
                    step stamps_rand 300 env TRX_DAMAGE=random python tools/phase_stamps.py 4096 &&
                    step stamps_rand_reset 300 env TRX_DAMAGE=random TRX_STAMP_RESET=1 python tools/phase_stamps.py 4096 ;;
        epw) for e in 1 2 3 4; do step bench_epw$e 300 env TRX_EPW=$e python bench.py --workload env --steps 44 --warmup 22 --no-cpu; done ;;
        dettests) step det_tests 600 python -u -m pytest tests/test_determinism.py -m gpu -v -s --timeout 500 --timeout-method thread ;;
        gattests) step gat_tests 400 python -u -m pytest tests/test_gat_infer.py tests/test_gat.py tests/test_sac.py tests/test_gat_tail.py -m gpu -v --timeout 120 --timeout-method thread ;;
        actmid) TRX_MID=0 step act_mid0 300 rocprofv3 --kernel-trace --stats -d gpurun_out/act_mid0 -o run --output-format csv -- python3 tools/agent_profile.py 4096 act &&
                TRX_MID=1 step act_mid1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/act_mid1 -o run --output-format csv -- python3 tools/agent_profile.py 4096 act ;;
        act) step act 300 rocprofv3 --kernel-trace --stats -d gpurun_out/act -o run --output-format csv -- python3 tools/agent_profile.py 4096 act ;;
        upd) step upd 300 rocprofv3 --kernel-trace --stats -d gpurun_out/upd -o run --output-format csv -- python3 tools/agent_profile.py 4096 update ;;
        overlap) step overlap 300 python tools/overlap_probe.py 4096 ;;
        ehab) step eh_cs_a 200 env TRX_LIB=$PWD/sac-gat-her_transportationrl_amd/trafficrl/libtrafficrl_old.so python tools/act_checksum.py 4096 &&
              step eh_cs_b 200 python tools/act_checksum.py 4096 &&
              TRX_LIB=$PWD/sac-gat-her_transportationrl_amd/trafficrl/libtrafficrl_old.so step act_a 300 rocprofv3 --kernel-trace --stats -d gpurun_out/act_a -o run --output-format csv -- python3 tools/agent_profile.py 4096 act &&
              step act 300 rocprofv3 --kernel-trace --stats -d gpurun_out/act -o run --output-format csv -- python3 tools/agent_profile.py 4096 act ;;
        updactor) TRX_FP32_ACTOR=0 step upd_bf16actor 300 python tools/agent_profile.py 4096 update &&
                  TRX_FP32_ACTOR=1 step upd_fp32actor 300 python tools/agent_profile.py 4096 update ;;
        updstreams) TRX_UPD_STREAMS=2 step upd_s2 300 python tools/agent_profile.py 4096 update &&
                    TRX_UPD_STREAMS=3 step upd_s3 300 python tools/agent_profile.py 4096 update &&
                    TRX_UPD_STREAMS=6 step upd_s6 300 python tools/agent_profile.py 4096 update &&
                    TRX_UPD_STREAMS=1 step upd_s1 300 python tools/agent_profile.py 4096 update ;;
        updserial) step upd_default 300 python tools/agent_profile.py 4096 update &&
                   TRX_UPD_SERIAL=fwd step upd_fwdserial 300 python tools/agent_profile.py 4096 update ;;
        hwq) for q in 4 8 16; do GPU_MAX_HW_QUEUES=$q step upd_q$q 300 python tools/agent_profile.py 4096 update || exit 1; done
             DEBUG_HIP_FORCE_GRAPH_QUEUES=6 step upd_gq6 300 python tools/agent_profile.py 4096 update &&
             DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 step upd_nopc 300 python tools/agent_profile.py 4096 update &&
             step upd_log 300 bash -c "AMD_LOG_LEVEL=3 python tools/agent_profile.py 4096 update 2>&1 | grep -a -m 20 -E 'parallel streams|update wall'" ;;
        bigab) L=$PWD/sac-gat-her_transportationrl_amd/trafficrl/libtrafficrl.so
               step abbig_a 300 python tools/ab_big.py $L 1024 && step abbig_b 300 python tools/ab_big.py $L 1024 &&
               step profana 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profana -o run --output-format csv -- python3 bench.py --network anaheim --steps 6 --warmup 2 --no-cpu ;;
        poolab) step fused_tests 600 python -u -m pytest tests/test_split_gemm.py tests/test_fused_update.py tests/test_sac_e2e.py tests/test_sac.py tests/test_gat_infer.py tests/test_gat.py tests/test_gat_tail.py -m gpu -x -q --timeout 300 --timeout-method thread ;;
        perov) step per_tests 400 python -u -m pytest tests/test_per_tree.py tests/test_replay_train.py tests/test_determinism.py -m gpu -x -q --timeout 300 --timeout-method thread &&
               TRX_PER_OVERLAP=0 step bench_pov0 400 python bench.py --steps 44 --warmup 22 --no-cpu && step bench_pov1 400 python bench.py --steps 44 --warmup 22 --no-cpu &&
               TRX_PER_OVERLAP=0 step bench_pov0b 400 python bench.py --steps 44 --warmup 22 --no-cpu && step bench_pov1b 400 python bench.py --steps 44 --warmup 22 --no-cpu ;;
        updtl) step updtl 300 rocprofv3 --kernel-trace -d gpurun_out/updtl -o run --output-format csv -- python3 tools/upd_timeline.py run &&
               python tools/upd_timeline.py report $(ls gpurun_out/updtl/*/run_kernel_trace.csv gpurun_out/updtl/run_kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/updtl_report.txt 2>&1 ;;
        multi2) for m in 0 1 2; do TRX_UPD_MULTI=$m step upd_time_m$m 300 python tools/upd_time.py || exit 1; done &&
                for m in 1 2; do TRX_UPD_MULTI=$m step updtl_m$m 300 rocprofv3 --kernel-trace -d gpurun_out/updtl_m$m -o run --output-format csv -- python3 tools/upd_timeline.py run || exit 1
                    python tools/upd_timeline.py report $(ls gpurun_out/updtl_m$m/*/run_kernel_trace.csv gpurun_out/updtl_m$m/run_kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/updtl_m${m}_report.txt 2>&1; done ;;
        prio) step prio_tests 900 python -u -m pytest tests/test_replay_train.py tests/test_determinism.py tests/test_concurrent_update.py tests/test_per_tree.py tests/test_fused_update.py -m gpu -x -v --timeout 300 --timeout-method thread &&
              step upd_time_prio 300 python tools/upd_time.py ;;
        adam) step adam_tests 600 python -u -m pytest tests/test_flat_adam.py tests/test_replay_train.py tests/test_determinism.py -m gpu -x -v --timeout 300 --timeout-method thread &&
              step upd_time_adam 300 python tools/upd_time.py &&
              step updtl 300 rocprofv3 --kernel-trace -d gpurun_out/updtl -o run --output-format csv -- python3 tools/upd_timeline.py run &&
              python tools/upd_timeline.py report $(ls gpurun_out/updtl/*/run_kernel_trace.csv gpurun_out/updtl/run_kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/updtl_report.txt 2>&1 ;;
        fmatests) step fma_tests 900 python -u -m pytest tests/test_gat_infer.py tests/test_gat_tail.py tests/test_sac_e2e.py tests/test_fused_update.py tests/test_gat.py tests/test_sac.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
        wsplit) step wsplit 300 python tools/wgrad3_split.py ;;
        updab) for r in 1 2; do for L in libtrafficrl libtrafficrl_${VAR:-x}; do TRX_LIB=sac-gat-her_transportationrl_amd/trafficrl/$L.so step upd_ab_${L}_$r 300 python tools/upd_time.py || exit 1; echo "$L $(tail -1 gpurun_out/upd_ab_${L}_$r.log)" >> gpurun_out/updab_summary.txt; done; done ;;
        actab) T=sac-gat-her_transportationrl_amd/trafficrl
               for r in 1 2; do for L in libtrafficrl libtrafficrl_${VAR:-x}; do
                   TRX_LIB=$T/$L.so step actab_${L}_$r 300 rocprofv3 --kernel-trace --stats -d gpurun_out/actab_${L}_$r -o run --output-format csv -- python3 tools/agent_profile.py 4096 act || exit 1; done; done ;;
        disttests) step dist_tests 600 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
        dist2) step bench_dist2 600 env TRX_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 44 --warmup 22 --no-cpu ;;
        branchprobe) step branch_probe3 300 python tools/branch_probe.py 3 && step branch_probe6 300 python tools/branch_probe.py 6 ;;
        fu1) step fu1 150 env AMD_SERIALIZE_KERNEL=3 python -u -m pytest tests/test_fused_update.py -m gpu -x -v -s --timeout 60 --timeout-method thread -k vs_fp32_restatement ;;
        mprobe) step multi_probe 150 python -u tools/multi_probe.py 5 && PROBE_STAGES=1 step multi_stages 150 python -u tools/multi_probe.py 5 ;;
        multi) step multi_tests 900 python -u -m pytest tests/test_fused_update.py tests/test_concurrent_update.py tests/test_sac_e2e.py tests/test_gat_infer.py tests/test_flat_adam.py -m gpu -x -v -s --timeout 300 --timeout-method thread &&
               TRX_UPD_MULTI=0 step upd_time_m0 300 python tools/upd_time.py && TRX_UPD_MULTI=1 step upd_time_m1 300 python tools/upd_time.py &&
               TRX_UPD_MULTI=0 step upd_time_m0b 300 python tools/upd_time.py && TRX_UPD_MULTI=1 step upd_time_m1b 300 python tools/upd_time.py ;;
        resab) step gat_e2e 600 python -u -m pytest tests/test_gat_infer.py tests/test_sac_e2e.py tests/test_gat_tail.py tests/test_capi_cpu.py -m gpu -v -s --timeout 300 --timeout-method thread &&
               TRX_RES_BF16=0 step act_res0 300 python tools/agent_profile.py 4096 act && TRX_RES_BF16=1 step act_res1 300 python tools/agent_profile.py 4096 act &&
               TRX_RES_BF16=0 step act_res0b 300 python tools/agent_profile.py 4096 act && TRX_RES_BF16=1 step act_res1b 300 python tools/agent_profile.py 4096 act ;;
        updt) step upd_time 300 python tools/upd_time.py ;;
        walls) step walls_act 300 python tools/agent_profile.py 4096 act && step walls_upd 300 python tools/agent_profile.py 4096 update ;;
        istamps) step istamps 300 python tools/infer_stamps.py 4096 ;;
        abact) TRX_LIB=${TRX_LIB_A:-} step act_a 300 rocprofv3 --kernel-trace --stats -d gpurun_out/act_a -o run --output-format csv -- python3 tools/agent_profile.py 4096 act
               TRX_LIB=sac-gat-her_transportationrl_amd/trafficrl/libtrafficrl_old.so step act_b 300 rocprofv3 --kernel-trace --stats -d gpurun_out/act_b -o run --output-format csv -- python3 tools/agent_profile.py 4096 act ;;
        abk) step ab_quad 200 env TRX_KERNEL=quad python tools/ab_env.py sac-gat-her_transportationrl_amd/trafficrl/libtrafficrl.so 4096 30 ;;
        fused) step fused_tests 600 python -u -m pytest tests/test_split_gemm.py tests/test_flat_adam.py tests/test_fused_update.py tests/test_sac_e2e.py tests/test_sac.py -m gpu -v -s --timeout 300 --timeout-method thread ;;
        bigstats) step big_stats 300 python tools/big_stats.py 1024 fw ;;
        actab) for f in sac-gat-her_transportationrl_amd/trafficrl/libtrafficrl.so sac-gat-her_transportationrl_amd/trafficrl/libtrafficrl_l03.so; do [ -f $f ] || continue; n=$(basename $f .so); TRX_LIB=$PWD/$f step actab_$n 200 python tools/act_host_probe.py 4096 || exit 1; done
               grep -h "eager" gpurun_out/actab_*.log ;;
        actprobe) step act_probe 300 python tools/act_host_probe.py 4096 ;;
        graphtests) step graph_tests 400 python -u -m pytest tests/test_replay_train.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
        fallback) step fallback_tests 400 python -u -m pytest tests/test_gpu_fallback.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
        abt) for f in sac-gat-her_transportationrl_amd/trafficrl/libtrafficrl*.so; do n=$(basename $f .so); step abt_$n 200 python tools/ab_env.py $f 4096 20 torch || exit 1; done ;;
        abo) for f in sac-gat-her_transportationrl_amd/trafficrl/libtrafficrl*.so; do n=$(basename $f .so); step abo_$n 200 python tools/ab_env.py $f 4096 30 obs || exit 1; done ;;
        abv) for f in sac-gat-her_transportationrl_amd/trafficrl/libtrafficrl*.so; do n=$(basename $f .so); case $n in *stamps*) continue;; esac; step ab_$n 200 python tools/ab_env.py $f 4096 30 || exit 1; done
             grep -h "step kernel" gpurun_out/ab_*.log ;;
        vtest) cp sac-gat-her_transportationrl_amd/trafficrl/libtrafficrl_${VARIANT}.so $LIB && sha256sum $LIB | cut -c1-16 > gpurun_out/lib_sha16.txt
               step vtest_$VARIANT 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sparse.py tests/test_gpu_fallback.py tests/test_torch_sp.py tests/test_gpu_large.py -m gpu -x -q --timeout 300 --timeout-method thread ;;
        abbig) for f in sac-gat-her_transportationrl_amd/trafficrl/libtrafficrl*.so; do n=$(basename $f .so); case $n in *stats*|*stamps*) continue;; esac; step abbig_$n 200 python tools/ab_big.py $f 1024 || exit 1; done
               grep -h "step kernel" gpurun_out/abbig_*.log ;;
        abx) for f in sac-gat-her_transportationrl_amd/trafficrl/libtrafficrl*.so; do n=$(basename $f .so); step ab_$n 200 python tools/ab_env.py $f 4096 30 || exit 1; done ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done


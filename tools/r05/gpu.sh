# Round-5 GPU calls: one stage per gpurun call, `bash tools/r05/gpu.sh <stage>`,
# run from the repository root on the GPU box.  Every GPU step has its own time
# limit and the steps are chained with &&, so the first failure ends the call.
# Outputs go to gpurun_out/r05<stage>/; the ones kept are copied to
# profiles/r05/r05<stage>/.  (One indexed file instead of round 4's one script
# per call; the stage letter is the record's name.)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
S=$1; O=gpurun_out/r05$S; mkdir -p $O
pt() {  # name, seconds, pytest args...
  local n=$1 s=$2; shift 2
  timeout -k 10 $s python -u -m pytest -x -v --timeout 600 --timeout-method thread "$@" > $O/pytest_$n.txt 2>&1
}
b() {  # name, seconds, bench args...
  local n=$1 s=$2; shift 2
  timeout -k 10 $s python -u bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.log
}
E=first_raytracer_amd/build/exp
ab() {  # tag, lib ('' = in-tree), perf_ab args...
  local t=$1 l=$2; shift 2
  if [ -n "$l" ]; then FRT_LIB_PATH=$E/$l timeout -k 10 300 python -u tools/perf_ab.py "$@" >> $O/ab_$t.jsonl 2>> $O/ab.log
  else timeout -k 10 300 python -u tools/perf_ab.py "$@" >> $O/ab_$t.jsonl 2>> $O/ab.log; fi
}
C="--scene cornell --spp 512 --rounds 3 --bvh gsah --variants default"
P="--scene cornell --spp 512 --rounds 2 --bvh gsah --integrator pssmlt --variants default"
M="--scene cornell_1m --spp 256 --rounds 2 --bvh gsah --variants default"
case $S in
a)  # the GPU suite (C5 chain-shard parity is new) + smoke on the build with
    # octant-plan pop culling and the octant plan for PSS-MLT, then the PSS-MLT line
    pt gpu 1100 tests -m gpu \
     && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
     && b pssmlt 500 --integrator pssmlt ;;
b)  # (ran with the diag build's PSS-MLT bootstrap ticking into an unset
    # buffer: GPU fault in diag_mlt, fixed in the next build; the default and
    # gloo2 lines above it completed)
    b default 500 \
     && b gloo2 400 --gpus 2 --backend gloo --steps 2 --north-star off \
     && FRT_LIB_PATH=$E/libfrt_diag.so timeout -k 10 200 python tools/diag_phases.py --scene cornell --spp 32 > $O/diag_cornell.json 2> $O/diag.log \
     && FRT_LIB_PATH=$E/libfrt_diag.so timeout -k 10 200 python tools/diag_phases.py --scene cornell --integrator pssmlt --spp 64 > $O/diag_mlt.json 2>> $O/diag.log ;;
c)  # same-call A/B: in-tree (octant + 4-wide pop culling, 7-word items, 15-entry
    # 4-wide LDS stack, PSS-MLT on the octant plan) / nocull (the same without
    # the entry-distance tests) / cull2 (octant culling + PSS-MLT octant plan,
    # 10-word items) / base (round-5 start); then the diagnostic build (path and
    # PSS-MLT) and the parity tests of the in-tree build
    for k in 1 2; do ab c "" $C && ab c libfrt_nocull.so $C && ab c libfrt_cull2.so $C && ab c libfrt_base.so $C || exit 1; done \
     && for k in 1 2; do ab m "" $M && ab m libfrt_nocull.so $M && ab m libfrt_base.so $M || exit 1; done \
     && for k in 1 2; do ab mlt "" $P && ab mlt libfrt_base.so $P || exit 1; done \
     && FRT_LIB_PATH=$E/libfrt_diag.so timeout -k 10 200 python tools/diag_phases.py --scene cornell --spp 32 > $O/diag_cornell.json 2> $O/diag.log \
     && FRT_LIB_PATH=$E/libfrt_diag.so timeout -k 10 200 python tools/diag_phases.py --scene cornell --integrator pssmlt --spp 64 > $O/diag_mlt.json 2>> $O/diag.log \
     && FRT_LIB_PATH=$E/libfrt_diag.so timeout -k 10 200 python tools/diag_phases.py --scene cornell_1m --spp 32 > $O/diag_1m.json 2>> $O/diag.log \
     && pt parity 600 tests/test_gpu_parity.py tests/test_gpu_c4.py tests/test_gpu_trace.py tests/test_gpu_pssmlt.py -m gpu ;;
d)  # same-call A/B of the node-or-leaf ("if-if") loop on the octant plan
    # (ifif20 / ifif8: the wave leaves at 20 / 8 working lanes) against the
    # in-tree descend-then-test step, on Cornell and PSS-MLT; PSS-MLT trav_min
    for k in 1 2; do ab c "" $C && ab c libfrt_ifif20.so $C && ab c libfrt_ifif8.so $C || exit 1; done \
     && for k in 1 2; do ab mlt "" $P && ab mlt libfrt_ifif20.so $P && ab mlt libfrt_ifif8.so $P || exit 1; done \
     && ab mltt "" --scene cornell --spp 512 --rounds 2 --bvh gsah --integrator pssmlt \
          --variants default,default/trav6,default/trav20,default/trav28,default ;;
e)  # the build after the round's A/Bs (pop culling, 7-word items, if-if
    # removed; PSS-MLT on the octant plan): GPU suite + smoke, the PSS-MLT
    # line under rocprofv3 kernel-trace + stats, its three PMC passes
    SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
    pmc() {  # name, counters, bench args...
      local n=$1 c=$2; shift 2
      timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/$n -o run -- \
          python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --north-star off "$@" > $O/$n.json 2> $O/$n.log
    }
    pt gpu 900 tests -m gpu \
     && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
     && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_pssmlt -o run -- \
          python3 bench.py --integrator pssmlt --steps 3 --warmup 1 > $O/bench_pssmlt.json 2> $O/bench_pssmlt.log \
     && pmc sq_pssmlt "$SQ" --integrator pssmlt && pmc fetch_pssmlt FETCH_SIZE --integrator pssmlt \
     && pmc write_pssmlt WRITE_SIZE --integrator pssmlt ;;
f)  # same-call A/B: the compiler's SLP vectorizer off (-fno-slp-vectorize, build/exp/libfrt_noslp.so),
    # and on cornell_1m the BVH4Q planes as fp16 for v_fma_mix_f32 (libfrt_f16.so, FRT_F16_PLANES=1),
    # against the in-tree build (libfrt_cur.so, identical to it): the vectorizer packs float pairs
    # into v_pk_* with register moves around them (115 v_pk / 233 v_mov in the cornell_1m kernel;
    # without: 0 / 168, 20 -> 5 scratch instructions, Cornell 12 -> 0)
    V="--scene veach --spp 256 --rounds 2 --variants default"
    for k in 1 2; do ab c libfrt_cur.so $C && ab c libfrt_noslp.so $C || exit 1; done \
     && for k in 1 2; do ab m libfrt_cur.so $M && ab m "" $M && ab m libfrt_noslp.so $M && ab m libfrt_f16.so $M && ab m libfrt_f16noslp.so $M || exit 1; done \
     && for k in 1 2; do ab mlt libfrt_cur.so $P && ab mlt libfrt_noslp.so $P || exit 1; done \
     && for k in 1 2; do ab v libfrt_cur.so $V && ab v libfrt_noslp.so $V || exit 1; done ;;
g)  # the build with -fno-slp-vectorize: GPU suite (incl. the register-cap tables, whose kernels the
    # flag recompiled) + smoke, then tools/gpu_roofline.sh part a: the default bench line under
    # rocprofv3 kernel-trace + stats and the Cornell / cornell_1m PMC passes
    pt gpu 900 tests -m gpu \
     && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
     && TAG=r05$S PART=a STEPS=5 timeout -k 10 900 bash tools/gpu_roofline.sh > $O/roofline.log 2>&1 ;;
h)  # tools/gpu_roofline.sh part b: veach and PSS-MLT lines under rocprofv3, their PMC passes
    TAG=r05$S PART=b timeout -k 10 1000 bash tools/gpu_roofline.sh > $O/roofline.log 2>&1 ;;
i)  # same-call A/B on the -fno-slp-vectorize build (libfrt_cur.so = in-tree): the machine
    # scheduler's max-ilp and max-memory-clause strategies (libfrt_ilp / _memclause), and a 7-wave
    # HBM plan (libfrt_w7: 12 LDS stack entries, 22 KiB a block, the 6-wave plans capped at 7)
    for k in 1 2; do ab c libfrt_cur.so $C && ab c libfrt_ilp.so $C && ab c libfrt_memclause.so $C || exit 1; done \
     && for k in 1 2; do ab m libfrt_cur.so $M && ab m libfrt_ilp.so $M && ab m libfrt_memclause.so $M && ab m libfrt_w7.so $M || exit 1; done \
     && for k in 1 2; do ab mlt libfrt_cur.so $P && ab mlt libfrt_ilp.so $P && ab mlt libfrt_memclause.so $P || exit 1; done ;;
j)  # the build with the 7-wave 4-wide HBM plan: GPU suite + smoke, the default line (Cornell +
    # north star), the PSS-MLT line with its path-exact parity and CPU baseline
    pt gpu 900 tests -m gpu \
     && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
     && b default 500 && b pssmlt 500 --integrator pssmlt ;;
k)  # PMC on the final kernels: the 7-wave cornell_1m plan (bench --scene cornell_1m), AO and
    # normals (their bench lines under rocprofv3 kernel-trace first)
    SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
    pmc() {  # name, counters, bench args...
      local n=$1 c=$2; shift 2
      timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/$n -o run -- \
          python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --north-star off "$@" > $O/$n.json 2> $O/$n.log
    }
    tr() {  # name, bench args...
      local n=$1; shift
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$n -o run -- \
          python3 bench.py "$@" > $O/trace_$n.json 2> $O/trace_$n.log
    }
    pmc sq_1m "$SQ" --scene cornell_1m && pmc fetch_1m FETCH_SIZE --scene cornell_1m \
     && pmc write_1m WRITE_SIZE --scene cornell_1m && pmc tcc_1m "TCC_HIT TCC_MISS" --scene cornell_1m \
     && tr ao --integrator ao --steps 5 --warmup 1 && tr normals --integrator normals --steps 5 --warmup 1 \
     && pmc sq_ao "$SQ" --integrator ao && pmc fetch_ao FETCH_SIZE --integrator ao && pmc write_ao WRITE_SIZE --integrator ao \
     && pmc sq_normals "$SQ" --integrator normals && pmc fetch_normals FETCH_SIZE --integrator normals \
     && pmc write_normals WRITE_SIZE --integrator normals ;;
l)  # same-call A/B: 9-word work items (the linear pixel index derived; libfrt_item9) so that a
    # 6th 26-KiB octant block fits a CU, at the default 5-wave and the 6-wave cap, against the
    # in-tree build (libfrt_cur); cornell_1m as a check (7 waves either way); the PSS-MLT chain
    # kernel at a 5-wave cap (libfrt_mlt5; 105 VGPRs uncapped since the SLP vectorizer is off)
    C6="--scene cornell --spp 512 --rounds 3 --bvh gsah --variants default,waves6"
    for k in 1 2; do ab c libfrt_cur.so $C6 && ab c libfrt_item9.so $C6 || exit 1; done \
     && for k in 1 2; do ab m libfrt_cur.so $M && ab m libfrt_item9.so $M || exit 1; done \
     && for k in 1 2; do ab mlt libfrt_cur.so $P && ab mlt libfrt_mlt5.so $P || exit 1; done ;;
m)  # the N-way split's load balance on the final kernels (each shard alone on the GPU), Cornell
    # and cornell_1m at 1080p 512 spp
    timeout -k 10 500 python -u tools/shard_balance.py --scene cornell --ns 2,4,8 --reps 2 > $O/shard_cornell.json 2> $O/shard.log \
     && timeout -k 10 600 python -u tools/shard_balance.py --scene cornell_1m --ns 2,4,8 --reps 1 > $O/shard_1m.json 2>> $O/shard.log ;;
n)  # final-build check: GPU suite + smoke, the default line, veach line, and the launcher's
    # two-rank gloo rehearsal (one GPU) with the north-star block
    pt gpu 900 tests -m gpu \
     && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
     && b default 500 && b veach 400 --scene veach --spp 1024 \
     && b gloo2 600 --gpus 2 --backend gloo --steps 2 ;;
o)  # same-call A/B on cornell_1m: unconditional pushes above the 4-wide stack top (libfrt_pushu)
    # against the in-tree build (libfrt_cur)
    for k in 1 2; do ab m libfrt_cur.so $M && ab m libfrt_pushu.so $M || exit 1; done ;;
p)  # rocprofv3 kernel-trace + stats of the default bench command on the final build (the launch
    # averages the line's roofline divides by)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_default -o run -- \
        python3 bench.py > $O/trace_default.json 2> $O/trace_default.log ;;
q)  # scheduling knobs re-checked on the final build: Cornell trav_min (default 20), cornell_1m
    # trav_min / min_desc (defaults 40 / 12) at the 7-wave plan
    ab ct "" --scene cornell --spp 512 --rounds 3 --bvh gsah --variants default,default/trav12,default/trav16,default/trav24,default/trav28,default \
     && ab mt "" --scene cornell_1m --spp 256 --rounds 2 --bvh gsah --variants default,default/trav32,default/trav48,default/desc8,default/desc16,default ;;
r)  # same-call A/B on cornell_1m: an 8-wave 4-wide HBM plan (libfrt_w8: 10 LDS stack entries,
    # 20 KiB a block, eight to a CU; 64 VGPRs, 25 spilled) against the in-tree 7-wave plan
    for k in 1 2; do ab m "" $M && ab m libfrt_w8.so $M || exit 1; done ;;
s)  # same-call A/B on cornell_1m: the area-optimal 4-wide collapse (libfrt_dp, FRT_EXP_BVH4_DP=1:
    # per binary node the least summed node area over 1..4 slots; host SAH tree 148603 -> 113784
    # nodes, node area sum -1.5 %) against the in-tree greedy collapse
    for k in 1 2; do ab m "" $M && ab m libfrt_dp.so $M || exit 1; done ;;
t)  # the build with the area-optimal 4-wide collapse: GPU suite + smoke, the default line
    pt gpu 900 tests -m gpu \
     && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
     && b default 500 ;;
u)  # the area-optimal collapse build: cornell_1m PMC passes (bench --scene cornell_1m), then the
    # default bench command under rocprofv3 kernel-trace + stats
    SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
    pmc() {  # name, counters, bench args...
      local n=$1 c=$2; shift 2
      timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/$n -o run -- \
          python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --north-star off "$@" > $O/$n.json 2> $O/$n.log
    }
    pmc sq_1m "$SQ" --scene cornell_1m && pmc fetch_1m FETCH_SIZE --scene cornell_1m \
     && pmc write_1m WRITE_SIZE --scene cornell_1m && pmc tcc_1m "TCC_HIT TCC_MISS" --scene cornell_1m \
     && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_default -o run -- \
          python3 bench.py > $O/trace_default.json 2> $O/trace_default.log ;;
v)  # same-call A/B on cornell_1m: SAH-terminated leaves of up to 8 triangles (libfrt_lsah,
    # FRT_EXP_LEAF_SAH=1; FRT_LEAF_SAH = 100 x triangle / binary-node cost) against the in-tree
    # "every subtree of <= 4 triangles" rule.  Host SAH tree: mean leaf 3.45 (in-tree), 6.27 / 4.63 /
    # 3.18 at 20 / 35 / 50
    M8="--scene cornell_1m --spp 256 --rounds 2 --bvh gsah --variants default/leaf8"
    for k in 1 2; do ab m "" $M && for r in 28 35 42 50; do FRT_LEAF_SAH=$r ab m$r libfrt_lsah.so $M8 || exit 1; done || exit 1; done ;;
w)  # leaf size on the LDS octant plan (default 2), Cornell and PSS-MLT, same call
    ab cl "" --scene cornell --spp 512 --rounds 3 --bvh gsah --variants default,default/leaf1,default/leaf3,default/leaf4,default \
     && ab mltl "" --scene cornell --spp 512 --rounds 2 --bvh gsah --integrator pssmlt --variants default,default/leaf1,default/leaf3,default ;;
x)  # same-call A/B: the binary traversal's stack top in a register (libfrt_topreg,
    # FRT_EXP_TOPREG=1: a pop hands the top over at once and refills it from LDS off the critical
    # path) against the in-tree build, Cornell and PSS-MLT; then the parity tests on that library
    for k in 1 2; do ab c "" $C && ab c libfrt_topreg.so $C || exit 1; done \
     && for k in 1 2; do ab mlt "" $P && ab mlt libfrt_topreg.so $P || exit 1; done \
     && FRT_LIB_PATH=$E/libfrt_topreg.so pt parity 600 tests/test_gpu_parity.py tests/test_gpu_pssmlt.py -m gpu ;;
y)  # where the Cornell kernel's cycles go: the wave-cycle buckets (WAIT_ANY + WAIT_INST_ANY +
    # ACTIVE_INST_ANY = WAVE_CYCLES) and the instruction mix, two SQ passes (counters the box
    # lists only); cornell_1m pass A too
    timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
    have() { local out=""; for c in "$@"; do grep -qw "$c" $O/counters.txt && out="$out $c"; done; echo $out; }
    A=$(have SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS)
    B=$(have SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM)
    echo "A: $A" > $O/sets.txt; echo "B: $B" >> $O/sets.txt
    pmc() {  # name, counters, bench args...
      local n=$1 c=$2; shift 2
      timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/$n -o run -- \
          python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --north-star off "$@" > $O/$n.json 2> $O/$n.log
    }
    pmc sqa_cornell "$A" && pmc sqb_cornell "$B" && pmc sqa_1m "$A" --scene cornell_1m ;;
z)  # same-call A/B of the octant node step without branches (SQ_INSTS_SALU is 48 % of SQ_INSTS_VALU
    # on Cornell, r05y): libfrt_bf1 (store above the top and read below it every visit, selects
    # only), libfrt_bf2 (the store only; the pop keeps its branch); then parity on bf1
    for k in 1 2; do ab c "" $C && ab c libfrt_bf1.so $C && ab c libfrt_bf2.so $C || exit 1; done \
     && for k in 1 2; do ab mlt "" $P && ab mlt libfrt_bf1.so $P && ab mlt libfrt_bf2.so $P || exit 1; done \
     && FRT_LIB_PATH=$E/libfrt_bf1.so pt parity 600 tests/test_gpu_parity.py tests/test_gpu_pssmlt.py -m gpu ;;
aa) # the build with the node-visit forms (path / ray queries: kStepStore, PSS-MLT: kStepSelect):
    # GPU suite + smoke, same-call A/B against the previous build (libfrt_prev), the default line
    pt gpu 900 tests -m gpu \
     && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
     && for k in 1 2; do ab c libfrt_prev.so $C && ab c "" $C || exit 1; done \
     && for k in 1 2; do ab mlt libfrt_prev.so $P && ab mlt "" $P || exit 1; done \
     && b default 500 ;;
ab) # control experiment: 16 more LDS bytes per octant node visit (libfrt_ldsx reads the next record's
    # first part and discards it) -- how much would fewer bytes per visit (fp16 planes) be worth?
    for k in 1 2; do ab c "" $C && ab c libfrt_ldsx.so $C || exit 1; done \
     && for k in 1 2; do ab mlt "" $P && ab mlt libfrt_ldsx.so $P || exit 1; done ;;
ac) # the octant records as fp16 planes in a scene frame + the refs, 32 B (libfrt_oct16; was 48 B +
    # 8 B of refs): the GPU suite on that library first (parity of every octant-plan test), then the
    # same-call A/B against the in-tree build on Cornell and PSS-MLT
    FRT_LIB_PATH=$E/libfrt_oct16.so pt gpu 900 tests -m gpu \
     && for k in 1 2; do ab c "" $C && ab c libfrt_oct16.so $C || exit 1; done \
     && for k in 1 2; do ab mlt "" $P && ab mlt libfrt_oct16.so $P || exit 1; done ;;
ad) # PMC per-ray figures of the kernels the node-visit forms changed (Cornell, PSS-MLT, AO, normals),
    # the PSS-MLT line under rocprofv3 kernel-trace, then the default line under kernel-trace
    SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
    pmc() {  # name, counters, bench args...
      local n=$1 c=$2; shift 2
      timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/$n -o run -- \
          python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --north-star off "$@" > $O/$n.json 2> $O/$n.log
    }
    tr() {  # name, seconds, bench args...
      local n=$1 s=$2; shift 2
      timeout -k 10 $s rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$n -o run -- \
          python3 bench.py "$@" > $O/trace_$n.json 2> $O/trace_$n.log
    }
    pmc sq_cornell "$SQ" && pmc fetch_cornell FETCH_SIZE && pmc write_cornell WRITE_SIZE \
     && pmc sq_pssmlt "$SQ" --integrator pssmlt && pmc fetch_pssmlt FETCH_SIZE --integrator pssmlt \
     && pmc write_pssmlt WRITE_SIZE --integrator pssmlt \
     && pmc sq_ao "$SQ" --integrator ao && pmc fetch_ao FETCH_SIZE --integrator ao && pmc write_ao WRITE_SIZE --integrator ao \
     && pmc sq_normals "$SQ" --integrator normals && pmc fetch_normals FETCH_SIZE --integrator normals \
     && pmc write_normals WRITE_SIZE --integrator normals \
     && tr pssmlt 400 --integrator pssmlt --steps 3 --warmup 1 --no-cpu-baseline --north-star off \
     && tr default 600 ;;
ae) # PSS-MLT trav_min re-checked on the branch-free node step (default 12); the AO and normals lines
    ab mltt "" --scene cornell --spp 512 --rounds 2 --bvh gsah --integrator pssmlt \
          --variants default,default/trav6,default/trav16,default/trav20,default \
     && b ao 300 --integrator ao && b normals 300 --integrator normals ;;
af) # AO / normals lines read slower after the node-visit forms (r05ae vs r05k): same-call A/B of the
    # path kernels with the branchy step (libfrt_pbranch) against the in-tree kStepStore, AO and normals
    A="--scene cornell --spp 512 --rounds 3 --bvh gsah --integrator ao --variants default"
    N="--scene cornell --spp 512 --rounds 3 --bvh gsah --integrator normals --variants default"
    for k in 1 2; do ab ao "" $A && ab ao libfrt_pbranch.so $A || exit 1; done \
     && for k in 1 2; do ab nrm "" $N && ab nrm libfrt_pbranch.so $N || exit 1; done ;;
ag) # the build with the per-integrator node step (path: Store, AO / normals / ray queries: Branch,
    # PSS-MLT: Select): GPU suite + smoke, AO / normals PMC passes and lines, the default line
    SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
    pmc() {  # name, counters, bench args...
      local n=$1 c=$2; shift 2
      timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/$n -o run -- \
          python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --north-star off "$@" > $O/$n.json 2> $O/$n.log
    }
    pt gpu 900 tests -m gpu \
     && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
     && pmc sq_ao "$SQ" --integrator ao && pmc fetch_ao FETCH_SIZE --integrator ao && pmc write_ao WRITE_SIZE --integrator ao \
     && pmc sq_normals "$SQ" --integrator normals && pmc fetch_normals FETCH_SIZE --integrator normals \
     && pmc write_normals WRITE_SIZE --integrator normals \
     && b ao 300 --integrator ao && b normals 300 --integrator normals && b default 500 ;;
ah) # C3 (veach, list world): the BVH over the list (culling only; trace_list) against the in-order scan
    # (FRT_LIST_BVH=0), same library, alternated; then the GPU suite on the list-BVH build
    V="--scene veach --spp 256 --rounds 2 --variants default"
    for k in 1 2; do ab v "" $V && FRT_LIST_BVH=0 ab vscan "" $V || exit 1; done \
     && pt gpu 900 tests -m gpu ;;
ai) # C3: the list scan's entry index and prim ref made wave-uniform (readfirstlane; libfrt_luni)
    V="--scene veach --spp 256 --rounds 2 --variants default"
    for k in 1 2; do ab v "" $V && ab v libfrt_luni.so $V || exit 1; done ;;
aj) # C3: the uniform list scan (libfrt_luni: readfirstlane index / ref) and with the fp64 records by
    # scalar loads from the constant address space (libfrt_luni2) against the in-tree scan
    V="--scene veach --spp 256 --rounds 2 --variants default"
    for k in 1 2; do ab v "" $V && ab v libfrt_luni.so $V && ab v libfrt_luni2.so $V || exit 1; done ;;
ak) # the build with the uniform list scan (scalar loads of the list's records): GPU suite + smoke,
    # the veach line (C3), its PMC passes (fp64 issue weights)
    SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
    F64="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64"
    pmc() {  # name, counters, bench args...
      local n=$1 c=$2; shift 2
      timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/$n -o run -- \
          python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --north-star off "$@" > $O/$n.json 2> $O/$n.log
    }
    pt gpu 900 tests -m gpu \
     && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
     && b veach 400 --scene veach --spp 1024 \
     && pmc sq_veach "$SQ" --scene veach --spp 1024 && pmc fetch_veach FETCH_SIZE --scene veach --spp 1024 \
     && pmc write_veach WRITE_SIZE --scene veach --spp 1024 && pmc f64_veach "$F64" --scene veach --spp 1024 \
     && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_veach -o run -- \
          python3 bench.py --scene veach --spp 1024 --steps 3 --warmup 1 --no-cpu-baseline --north-star off \
          > $O/trace_veach.json 2> $O/trace_veach.log ;;
al) # the fp64 list scan with the records through the constant address space (the r05aj libfrt_luni2
    # form; stage ak ran a helper-function form whose loads stayed vector loads): A/B against the
    # previous build (libfrt_prev), the GPU suite, the veach line
    V="--scene veach --spp 256 --rounds 2 --variants default"
    for k in 1 2; do ab v libfrt_prev.so $V && ab v "" $V || exit 1; done \
     && pt gpu 900 tests -m gpu && b veach 400 --scene veach --spp 1024 ;;
am) # C3: every load of the fp64 list scan scalar (libfrt_lsc: the list entry and all three vertex
    # records through the constant address space, base-pointer indexing) against the in-tree build
    # (the vertex records v1 / v2 and the sphere scalar, the entry and v0 vector)
    V="--scene veach --spp 256 --rounds 2 --variants default"
    for k in 1 2; do ab v "" $V && ab v libfrt_lsc.so $V || exit 1; done ;;
an) # the build with every fp64 list-scan load scalar: GPU suite + smoke, the veach line, its PMC
    # passes and kernel trace (stage ak's steps)
    SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
    F64="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64"
    pmc() {  # name, counters, bench args...
      local n=$1 c=$2; shift 2
      timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/$n -o run -- \
          python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --north-star off "$@" > $O/$n.json 2> $O/$n.log
    }
    pt gpu 900 tests -m gpu \
     && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
     && b veach 400 --scene veach --spp 1024 \
     && pmc sq_veach "$SQ" --scene veach --spp 1024 && pmc fetch_veach FETCH_SIZE --scene veach --spp 1024 \
     && pmc write_veach WRITE_SIZE --scene veach --spp 1024 && pmc f64_veach "$F64" --scene veach --spp 1024 \
     && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_veach -o run -- \
          python3 bench.py --scene veach --spp 1024 --steps 3 --warmup 1 --no-cpu-baseline --north-star off \
          > $O/trace_veach.json 2> $O/trace_veach.log ;;
ao) # C3: the fp64 list kernels at a 3-wave register cap (libfrt_f64w3) against the compiler's own
    # allocation (2 waves), on the scalar-load build
    V="--scene veach --spp 256 --rounds 2 --variants default"
    for k in 1 2; do ab v "" $V && ab v libfrt_f64w3.so $V || exit 1; done ;;
ap) # cornell_1m trees on the final kernels: GPU binned SAH (the bench default), host binned SAH, the
    # reference's create_bvh topology (full-sweep SAH, one-prim leaves before collapse)
    for k in 1 2; do ab mt "" --scene cornell_1m --spp 256 --rounds 2 --bvh gsah --variants default \
      && ab mt "" --scene cornell_1m --spp 256 --rounds 2 --bvh sah --variants default \
      && ab mt "" --scene cornell_1m --spp 256 --rounds 2 --bvh host --variants default || exit 1; done ;;
aq) # the octant plan's leaves with the straight-line triangle test (libfrt_ostr; round 4 measured
    # -2.4 % on Cornell before the SLP vectorizer was turned off), Cornell and PSS-MLT; Cornell trav_min
    # re-checked on the Store node step
    for k in 1 2; do ab c "" $C && ab c libfrt_ostr.so $C || exit 1; done \
     && for k in 1 2; do ab mlt "" $P && ab mlt libfrt_ostr.so $P || exit 1; done \
     && ab ct "" --scene cornell --spp 512 --rounds 3 --bvh gsah --variants default,default/trav16,default/trav24,default ;;
ar) # final build: GPU suite + smoke, the default line, the PSS-MLT line (path-exact chain-shard parity,
    # CPU baseline), and the launcher's two-rank gloo rehearsal
    pt gpu 900 tests -m gpu \
     && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
     && b default 500 && b pssmlt 600 --integrator pssmlt \
     && b gloo2 600 --gpus 2 --backend gloo --steps 2 ;;
as) # cornell_1m: the 4-wide plan's leaf loop with the next triangle's loads issued ahead of the
    # current test (libfrt_lpf; 8 VGPRs spilled at the 7-wave cap) against the in-tree serial loop
    for k in 1 2; do ab m "" $M && ab m libfrt_lpf.so $M || exit 1; done ;;
at) # PSS-MLT chain kernel at a 5-wave cap (libfrt_mlt5) on the branch-free node step, against the
    # in-tree 4-wave cap
    for k in 1 2; do ab mlt "" $P && ab mlt libfrt_mlt5.so $P || exit 1; done ;;
au) # the fp32 list kernels with the list scan's scalar loads: veach at fp32 (bench --precision fp32),
    # the previous build (libfrt_prev) and the in-tree build alternated, then the GPU suite
    VB="--scene veach --spp 256 --precision fp32 --steps 3 --warmup 1 --no-cpu-baseline --north-star off"
    for k in 1 2; do FRT_LIB_PATH=$E/libfrt_prev.so b v32prev$k 300 $VB && b v32cur$k 300 $VB || exit 1; done \
     && pt gpu 900 tests -m gpu ;;
av) # cornell_1m: the 4-wide stack's top in a register (libfrt_b4top: a pop hands the next node over at
    # once, the LDS read refills the register off the critical path; 12 VGPRs spilled at the 7-wave cap)
    for k in 1 2; do ab m "" $M && ab m libfrt_b4top.so $M || exit 1; done ;;
aw) # Cornell at N = 1: samples per work item (automatic: 9 on the LDS plan) against larger items
    ab cs "" --scene cornell --spp 512 --rounds 3 --bvh gsah --variants default,default/spi16,default/spi32,default/spi64,default ;;
ax) # PSS-MLT: the Kelemen perturbation as selects around one exp (in-tree) against the branches
    # (libfrt_prev), then the PSS-MLT GPU tests and the PSS-MLT line on the in-tree build
    for k in 1 2; do ab mlt libfrt_prev.so $P && ab mlt "" $P || exit 1; done \
     && pt mlt 600 tests/test_gpu_pssmlt.py -m gpu && b pssmlt 600 --integrator pssmlt ;;
ay) # final build (branch-free perturbation): GPU suite + smoke, PSS-MLT PMC passes and its line under
    # rocprofv3 kernel-trace
    SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
    pmc() {  # name, counters, bench args...
      local n=$1 c=$2; shift 2
      timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/$n -o run -- \
          python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --north-star off "$@" > $O/$n.json 2> $O/$n.log
    }
    pt gpu 900 tests -m gpu \
     && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
     && pmc sq_pssmlt "$SQ" --integrator pssmlt && pmc fetch_pssmlt FETCH_SIZE --integrator pssmlt \
     && pmc write_pssmlt WRITE_SIZE --integrator pssmlt \
     && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_pssmlt -o run -- \
          python3 bench.py --integrator pssmlt --steps 3 --warmup 1 --no-cpu-baseline --north-star off \
          > $O/trace_pssmlt.json 2> $O/trace_pssmlt.log ;;
*) echo "unknown stage $S"; exit 2 ;;
esac

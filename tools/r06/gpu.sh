# Round-6 GPU calls: one stage per gpurun call, `bash tools/r06/gpu.sh <stage>`,
# run from the repository root on the GPU box.  Every GPU step has its own time
# limit and the steps are chained with &&, so the first failure ends the call.
# Outputs go to gpurun_out/r06<stage>/; the ones kept are copied to
# profiles/r06/r06<stage>/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
S=$1; O=gpurun_out/r06$S; mkdir -p $O
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
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
WT="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
pmc() {  # name, counters, bench args...
  local n=$1 c=$2; shift 2
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/$n -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --north-star off --configs off "$@" > $O/$n.json 2> $O/$n.log
}
C="--scene cornell --spp 512 --rounds 3 --bvh gsah --variants default"
P="--scene cornell --spp 512 --rounds 2 --bvh gsah --integrator pssmlt --variants default"
M="--scene cornell_1m --spp 256 --rounds 2 --bvh gsah --variants default"
case $S in
a)  # round-6 start: GPU suite + smoke on the build with the plan-read scene_bytes and the
    # 44-entry 4-wide overflow stack, then the driver's default command (now with the c3 and
    # c5 blocks) exactly as the driver runs it
    pt gpu 900 tests -m gpu \
     && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
     && b default 600 --gpus 1 --steps 20 --warmup 5 ;;
b)  # PSS-MLT round-6 changes (fingerprint in LDS, integer splat conversion, materialisation
    # loads grouped by 4 trips): the PSS-MLT parity tests on the in-tree build, then a same-call
    # A/B against the round-5 source (libfrt_base.so) and the group sizes 1 and 2
    pt mlt 600 tests/test_gpu_pssmlt.py -m gpu \
     && for k in 1 2; do ab mlt "" $P && ab mlt libfrt_base.so $P && ab mlt libfrt_mg1.so $P && ab mlt libfrt_mg2.so $P || exit 1; done \
     && for k in 1 2; do ab m "" $M && ab m libfrt_base.so $M || exit 1; done ;;
c)  # stage b's variants were all ~3 % slower than round 5 (574 -> 590 ms): isolate the change.
    # none = all three off (11 chain words, the rest as round 5); fponly / splatonly / grouponly =
    # one change each; base = the round-5 source
    for k in 1 2; do for v in libfrt_base.so libfrt_none.so libfrt_fponly.so libfrt_splatonly.so libfrt_grouponly.so ""; do
        ab mlt "$v" $P || exit 1; done; done ;;
d)  # the N-rank path of the default command (C2 + north star + C3 + C5 blocks) rehearsed with two
    # ranks sharing the box's one GPU (gloo, host-staged collectives): the driver's SCALE run executes
    # this command at N = 2, 4, 8 with RCCL
    b gloo2 600 --gpus 2 --backend gloo --steps 2 --warmup 1 ;;
e)  # the final build's evidence: the default command under rocprofv3 kernel-trace + stats, then per
    # config the PMC passes tools/roofline_pmc.py reads (sq, fetch, write, wait; C4 + tcc, C3 + f64),
    # one counter group per run, and the per-ray table written under gpurun_out
    F64="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64"
    rp() {  # key, extra roofline_pmc args, bench args... (passes named <tag>_<group>)
      local key=$1 tag=$2 extra=$3; shift 3
      python tools/roofline_pmc.py $key --sq $O/${tag}_sq --fetch $O/${tag}_fetch --write $O/${tag}_write \
          --wait $O/${tag}_wait $extra --bench $O/${tag}_sq.json --copy-to $O/pmc --out $O/roofline_pmc.json >> $O/roofline.log 2>&1
    }
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_default -o run -- \
        python3 bench.py --steps 5 --warmup 1 > $O/trace_default.json 2> $O/trace_default.log \
     && cp profiles/roofline_pmc.json $O/roofline_pmc.json \
     && pmc c2_sq "$SQ" && pmc c2_fetch FETCH_SIZE && pmc c2_write WRITE_SIZE && pmc c2_wait "$WT" \
     && rp path:cornell:1920x1080 c2 "" \
     && pmc c4_sq "$SQ" --scene cornell_1m && pmc c4_fetch FETCH_SIZE --scene cornell_1m \
     && pmc c4_write WRITE_SIZE --scene cornell_1m && pmc c4_wait "$WT" --scene cornell_1m \
     && pmc c4_tcc "TCC_HIT TCC_MISS" --scene cornell_1m \
     && rp path:cornell_1m:1920x1080 c4 "--tcc $O/c4_tcc" \
     && pmc c3_sq "$SQ" --scene veach --spp 1024 && pmc c3_fetch FETCH_SIZE --scene veach --spp 1024 \
     && pmc c3_write WRITE_SIZE --scene veach --spp 1024 && pmc c3_wait "$WT" --scene veach --spp 1024 \
     && pmc c3_f64 "$F64" --scene veach --spp 1024 \
     && rp path:veach:1920x1080:fp64 c3 "--f64 $O/c3_f64" \
     && pmc c5_sq "$SQ" --integrator pssmlt && pmc c5_fetch FETCH_SIZE --integrator pssmlt \
     && pmc c5_write WRITE_SIZE --integrator pssmlt && pmc c5_wait "$WT" --integrator pssmlt \
     && rp pssmlt:cornell:1920x1080 c5 "" ;;
f)  # the node loop under a wave-uniform trip count (kStepUniform, libfrt_uni.so: path and chain
    # kernels) against the in-tree forms (Store / Select), then stage d's two-rank rehearsal
    # (round 6 later: in-tree = the octant LDS plan's lambertian kernels in their own unit under the
    # max-memory-clause scheduler; libfrt_nosplit.so = the same source with them in the main unit;
    # libfrt_uni.so = the wave-uniform node loop, built before the split)
    pt benchline 600 tests/test_gpu_bench_line.py -m gpu \
     && for k in 1 2; do ab c "" $C && ab c libfrt_nosplit.so $C && ab c libfrt_uni.so $C || exit 1; done \
     && for k in 1 2; do ab mlt "" $P && ab mlt libfrt_nosplit.so $P && ab mlt libfrt_uni.so $P || exit 1; done \
     && b gloo2 600 --gpus 2 --backend gloo --steps 2 --warmup 1 ;;
h)  # the machine scheduler's iterative strategies: for the octant unit (ldsit*: C2, C5) and, through
    # DEFS on every unit, for cornell_1m's 4-wide kernel in the main unit (allit*)
    for k in 1 2; do ab c "" $C && ab c libfrt_ldsitilp.so $C && ab c libfrt_ldsitmaxocc.so $C || exit 1; done \
     && for k in 1 2; do ab mlt "" $P && ab mlt libfrt_ldsitilp.so $P && ab mlt libfrt_ldsitmaxocc.so $P || exit 1; done \
     && for k in 1 2; do ab m "" $M && ab m libfrt_allitilp.so $M && ab m libfrt_allitmaxocc.so $M && ab m libfrt_allitminreg.so $M || exit 1; done ;;
i)  # 7-word work items (end and pixel coordinates derived; libfrt_item7) and with them a 15-entry
    # LDS stack for the 4-wide plan (22 KiB a block, still 7 to a CU; libfrt_item7ls15), against the
    # in-tree build (10-word items, 12 entries; PSS-MLT chains now in their own iterative-maxocc unit)
    for k in 1 2; do ab m "" $M && ab m libfrt_item7.so $M && ab m libfrt_item7ls15.so $M || exit 1; done \
     && for k in 1 2; do ab c "" $C && ab c libfrt_item7.so $C || exit 1; done \
     && for k in 1 2; do ab mlt "" $P || exit 1; done ;;
j)  # compiler flags per unit: AMDGPU register-pressure trackers in the scheduler (ldstrk: the octant
    # path unit only; alltrk: every unit), relaxed occupancy targets (allrelax: every unit), and the
    # material unit (C3's fp64 list kernel) under max-memory-clause / iterative-maxocc (matsmem,
    # matsmaxocc; it keeps the basic SGPR allocator)
    V="--scene veach --spp 256 --rounds 2 --variants default"
    for k in 1 2; do for v in "" libfrt_ldstrk.so libfrt_alltrk.so libfrt_allrelax.so; do ab c "$v" $C || exit 1; done; done \
     && for k in 1 2; do for v in "" libfrt_alltrk.so libfrt_allrelax.so; do ab m "$v" $M || exit 1; done; done \
     && for k in 1 2; do for v in "" libfrt_alltrk.so libfrt_allrelax.so; do ab mlt "$v" $P || exit 1; done; done \
     && for k in 1 2; do for v in "" libfrt_matsmem.so libfrt_matsmaxocc.so libfrt_alltrk.so libfrt_allrelax.so; do ab v "$v" $V || exit 1; done; done ;;
k)  # the final tree as the driver runs it: the GPU suite, smoke, then the default bench command
    pt gpu 900 tests -m gpu \
     && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
     && b default 600 --gpus 1 --steps 20 --warmup 5 ;;
l)  # full-frame parity (no sample, no estimate): C2 and C3 against the oracle on every pixel
    # (--rmse-min-frac 1), C5 path-exact on every chain of the frame (--mlt-shards 1)
    b c2full 600 --steps 3 --warmup 1 --north-star off --configs off --rmse-min-frac 1.0 \
     && b c3full 600 --scene veach --spp 1024 --steps 3 --warmup 1 --configs off --rmse-min-frac 1.0 \
     && b c5full 900 --integrator pssmlt --steps 3 --warmup 1 --mlt-shards 1 ;;
m)  # C4 (the north star) against the oracle on every pixel (~9 minutes of oracle on 16 threads)
    b c4full 1150 --scene cornell_1m --steps 3 --warmup 1 --configs off --rmse-min-frac 1.0 ;;
n)  # the unit-triangle (Woop) test in every fp32 kernel against Moller-Trumbore (knob removed after this A/B; needs the e32c42c sources)
    for k in 1 2; do ab c "" $C && ab c libfrt_woop.so $C || exit 1; done \
     && for k in 1 2; do ab mlt "" $P && ab mlt libfrt_woop.so $P || exit 1; done \
     && for k in 1 2; do ab m "" $M && ab m libfrt_woop.so $M || exit 1; done ;;
r)  # (record; the knob was removed after it) LDS-DMA touches on the 4-wide plan (FRT_EXP_TOUCH): the leaf's later lines (libfrt_touch.so),
    # the second-nearest child (libfrt_touchc.so), both (libfrt_touch3.so) vs the in-tree build:
    # cornell_1m 256 spp, then every library's film at a small size against the in-tree one
    F="--scene cornell_1m --spp 16 --res 480x270 --rounds 1 --variants default"
    for k in 1 2; do ab m "" $M && ab m libfrt_touch.so $M && ab m libfrt_touchc.so $M \
                     && ab m libfrt_touch3.so $M || exit 1; done \
     && timeout -k 10 300 python -u tools/perf_ab.py $F --save-films $O/films_base.npz > /dev/null 2>> $O/ab.log \
     && for l in touch touchc touch3; do FRT_LIB_PATH=$E/libfrt_$l.so timeout -k 10 300 python -u tools/perf_ab.py $F \
            --save-films $O/films_$l.npz > /dev/null 2>> $O/ab.log || exit 1; done \
     && python -c "import numpy as np; a=np.load('$O/films_base.npz'); print({l: bool(np.array_equal(a['default'], np.load('$O/films_'+l+'.npz')['default'])) for l in ('touch','touchc','touch3')})" > $O/films_equal.txt ;;
ac)  # (record; the knob was removed after it) the 4-wide leaf test two triangles a trip, their loads issued together (libfrt_pairs.so,
    # FRT_EXP_LEAF_PAIRS) vs the in-tree one-at-a-time loop: cornell_1m 256 spp, films of both
    F="--scene cornell_1m --spp 16 --res 480x270 --rounds 1 --variants default"
    for k in 1 2; do ab m "" $M && ab m libfrt_pairs.so $M || exit 1; done \
     && timeout -k 10 300 python -u tools/perf_ab.py $F --save-films $O/films_base.npz > /dev/null 2>> $O/ab.log \
     && FRT_LIB_PATH=$E/libfrt_pairs.so timeout -k 10 300 python -u tools/perf_ab.py $F --save-films $O/films_exp.npz > /dev/null 2>> $O/ab.log \
     && python -c "import numpy as np; a=np.load('$O/films_base.npz'); b=np.load('$O/films_exp.npz'); print({k: bool(np.array_equal(a[k], b[k])) for k in a.files})" > $O/films_equal.txt \
     && FRT_LIB_PATH=$E/libfrt_pairs.so pt c4 600 tests/test_gpu_c4.py tests/test_gpu_parity.py -m gpu -k "small_frame or bvh4 or config_spp" ;;
ab)  # short frames back to back in the bench's timed loop (~0.5 ms between launches): Cornell 1080p
    # at 64 spp, 20 steps, against perf_ab's launches with the film copied to the host in between
    b s64 300 --spp 64 --steps 20 --warmup 5 --configs off --north-star off --no-cpu-baseline \
     && timeout -k 10 300 python -u tools/perf_ab.py --scene cornell --spp 64 --rounds 5 --bvh gsah --variants default > $O/ab_s64.jsonl 2>> $O/ab.log ;;
aa)  # large frames: 4K at 512 spp and 8K at 128 spp on Cornell (the 32-bit queue, the partial-sum
    # workspace at 5.7 / 22 GB, RMSE on the bench's pixel sample), then 4K on cornell_1m
    b c4k 600 --res 3840x2160 --spp 512 --steps 3 --warmup 1 --configs off --north-star off \
     && b c8k 600 --res 7680x4320 --spp 128 --steps 2 --warmup 1 --configs off --north-star off \
     && b m4k 900 --scene cornell_1m --res 3840x2160 --spp 256 --steps 2 --warmup 1 --configs off --north-star off ;;
z)  # (record; the knob was removed after it) the octant node step's store deferred behind the next visit's record reads (libfrt_defer.so,
    # FRT_EXP_DEFER_PUSH) vs the in-tree build: Cornell 512 spp, PSS-MLT, then films of both libraries
    F1="--scene cornell --spp 16 --res 480x270 --rounds 1 --variants default"
    F2="--scene cornell --spp 16 --res 480x270 --rounds 1 --variants default --integrator pssmlt --chains 16384"
    for k in 1 2; do ab c "" $C && ab c libfrt_defer.so $C || exit 1; done \
     && for k in 1 2; do ab mlt "" $P && ab mlt libfrt_defer.so $P || exit 1; done \
     && timeout -k 10 300 python -u tools/perf_ab.py $F1 --save-films $O/fc_base.npz > /dev/null 2>> $O/ab.log \
     && FRT_LIB_PATH=$E/libfrt_defer.so timeout -k 10 300 python -u tools/perf_ab.py $F1 --save-films $O/fc_exp.npz > /dev/null 2>> $O/ab.log \
     && timeout -k 10 300 python -u tools/perf_ab.py $F2 --save-films $O/fm_base.npz > /dev/null 2>> $O/ab.log \
     && FRT_LIB_PATH=$E/libfrt_defer.so timeout -k 10 300 python -u tools/perf_ab.py $F2 --save-films $O/fm_exp.npz > /dev/null 2>> $O/ab.log \
     && python -c "import numpy as np; print({t: bool(np.array_equal(np.load('$O/f'+t+'_base.npz')['default'], np.load('$O/f'+t+'_exp.npz')['default'])) for t in 'cm'})" > $O/films_equal.txt ;;
y)  # the N = 8 code path rehearsed on one GPU: eight gloo ranks sharing the device (tile shards of
    # 1/8, the gather to rank 0, the PSS-MLT film sum, per_rank fields), the default blocks
    b gloo8 900 --gpus 8 --backend gloo --steps 2 --warmup 1 ;;
x)  # (record; the FRT_EXP_TIMELINE knob was removed after it) per-wave timeline of path_megakernel (libfrt_tl.so: entry, LDS scene loaded, first exhausted
    # queue grab, exit) at 64 and 512 spp, Cornell and cornell_1m
    FRT_LIB_PATH=$E/libfrt_tl.so timeout -k 10 400 python -u tools/r06/timeline.py > $O/timeline.jsonl 2> $O/timeline.log ;;
w)  # the per-launch fixed cost: Cornell and cornell_1m 1080p at 64 / 128 / 256 / 512 spp (time = a + b spp)
    for spp in 64 128 256 512; do
      timeout -k 10 300 python -u tools/perf_ab.py --scene cornell --spp $spp --rounds 3 --bvh gsah --variants default >> $O/spp_c.jsonl 2>> $O/ab.log || exit 1
    done \
     && for spp in 64 128 256 512; do
      timeout -k 10 300 python -u tools/perf_ab.py --scene cornell_1m --spp $spp --rounds 2 --bvh gsah --variants default >> $O/spp_m.jsonl 2>> $O/ab.log || exit 1
    done ;;
v)  # (record; the knob was removed after it) the fine tail (FRT_FINE_TAIL=1: the last chunk's samples cut into 8 chunks queued last): same
    # process at N = 1 (Cornell, cornell_1m), then every shard of N = 8 alone with and without it
    timeout -k 10 400 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 3 --bvh gsah \
        --variants default,default/fine1 > $O/ab_c.jsonl 2>> $O/ab.log \
     && timeout -k 10 400 python -u tools/perf_ab.py --scene cornell_1m --spp 512 --rounds 2 --bvh gsah \
        --variants default,default/fine1 > $O/ab_m.jsonl 2>> $O/ab.log \
     && timeout -k 10 300 python -u tools/shard_balance.py --scene cornell --ns 8 --reps 2 > $O/shard_cornell.json 2> $O/shard.log \
     && FRT_FINE_TAIL=1 timeout -k 10 300 python -u tools/shard_balance.py --scene cornell --ns 8 --reps 2 > $O/shard_cornell_fine.json 2>> $O/shard.log \
     && timeout -k 10 400 python -u tools/shard_balance.py --scene cornell_1m --ns 8 --reps 2 > $O/shard_1m.json 2>> $O/shard.log \
     && FRT_FINE_TAIL=1 timeout -k 10 400 python -u tools/shard_balance.py --scene cornell_1m --ns 8 --reps 2 > $O/shard_1m_fine.json 2>> $O/shard.log ;;
u)  # the N-way tile split on this round's kernels: every shard (r, N) timed alone on the GPU
    timeout -k 10 400 python -u tools/shard_balance.py --scene cornell --ns 2,4,8 --reps 2 > $O/shard_cornell.json 2> $O/shard.log \
     && timeout -k 10 500 python -u tools/shard_balance.py --scene cornell_1m --ns 2,4,8 --reps 2 > $O/shard_1m.json 2>> $O/shard.log ;;
t)  # the C4 GPU test at the configs' own sample counts (256 / 512 spp on 8,192 oracle pixels)
    pt c4 900 tests/test_gpu_c4.py -m gpu -k config_spp -s ;;
s)  # the AO and shading-normals integrators on this round's build (Cornell 1080p 512 spp lines)
    b ao 600 --integrator ao --steps 10 --warmup 3 --configs off --north-star off \
     && b normals 600 --integrator normals --steps 10 --warmup 3 --configs off --north-star off ;;
q)  # the clock each config's megakernel runs at (GRBM_GUI_ACTIVE over the dispatch, one pass per
    # config), merged into a copy of profiles/roofline_pmc.json (bench.py: clock_ghz,
    # valu_issue_frac_at_clock)
    CK="GRBM_GUI_ACTIVE GRBM_COUNT"
    cp profiles/roofline_pmc.json $O/roofline_pmc.json \
     && pmc c2_clk "$CK" && pmc c4_clk "$CK" --scene cornell_1m && pmc c3_clk "$CK" --scene veach --spp 1024 \
     && pmc c5_clk "$CK" --integrator pssmlt \
     && for x in "path:cornell:1920x1080 c2" "path:cornell_1m:1920x1080 c4" "path:veach:1920x1080:fp64 c3" \
                 "pssmlt:cornell:1920x1080 c5"; do set -- $x; \
          python tools/roofline_pmc.py $1 --clock $O/$2_clk --clock-only --copy-to $O/pmc --out $O/roofline_pmc.json \
              >> $O/roofline.log 2>&1 || exit 1; done ;;
p)  # the tree after the round's last experiments (sources as stage k's; bench.py with the
    # heartbeat and --mlt-shards): the GPU suite, smoke, the default bench command
    pt gpu 900 tests -m gpu \
     && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
     && b default 600 --gpus 1 --steps 20 --warmup 5 ;;
o)  # list-order records read one entry ahead in trace_list (libfrt_listrec.so) vs the in-tree scan:
    # veach 256 spp in fp64 (C3's kernel) and fp32, the films of both libraries, the C3 tests on it
    V="--scene veach --spp 256 --rounds 2 --variants default,fp32"
    F="--scene veach --spp 64 --res 480x270 --rounds 1 --variants default,fp32"
    for k in 1 2; do ab v "" $V && ab v libfrt_listrec.so $V || exit 1; done \
     && timeout -k 10 300 python -u tools/perf_ab.py $F --save-films $O/films_base.npz > /dev/null 2>> $O/ab.log \
     && FRT_LIB_PATH=$E/libfrt_listrec.so timeout -k 10 300 python -u tools/perf_ab.py $F --save-films $O/films_exp.npz > /dev/null 2>> $O/ab.log \
     && python -c "import numpy as np; a=np.load('$O/films_base.npz'); b=np.load('$O/films_exp.npz'); print({k: bool(np.array_equal(a[k], b[k])) for k in a.files})" > $O/films_equal.txt \
     && FRT_LIB_PATH=$E/libfrt_listrec.so pt veach 900 tests/test_gpu_precision.py -m gpu -k veach ;;
esac
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc

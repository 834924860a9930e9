#!/bin/bash
# Per-section shader-cycle profile of the path kernel (BDPT_PROF, bdpt_kernels.hip BDPT_TICK):
# one bench run per workload with a -DBDPT_PROF=1 specialised kernel and a fixed stream mode, so
# the profile holds one kernel kind.  Sections: s0 camera ray + closest hit, s1 hit shading,
# s2 NEE/VLP set-up and queue writes, s3 shadow rounds, s4 shadow results + contribution,
# s5 path end / accumulation / RNG loads.  The timer perturbs the kernel (s_memtime waits on
# lgkmcnt): shares, not speeds.  Output: gpurun_out/section_profile.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/section_profile.txt; : > "$out"
for spec in ${RUNS:-"cornell1080:64" "cornell1080:1" "weak64:32" "caustic8:1"}; do
    wl=${spec%%:*}; st=${spec##*:}
    echo "== $wl streams=$st" >> "$out"
    BDPT_PROF=1 BDPT_JIT_FLAGS="-DBDPT_PROF=1 ${EXTRA_FLAGS:-}" timeout -k 10 300 python bench.py --workload "$wl" \
        --streams "$st" --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/section_$wl.log 2>&1 || { echo "FAIL $wl $?"; exit 1; }
    grep bdpt_prof gpurun_out/section_$wl.log >> "$out"
    tail -1 gpurun_out/section_$wl.log | cut -c1-160 >> "$out"
done
cat "$out"

#!/bin/bash
# CPU side of scripts/profile_workloads.sh: turn its gpurun_out/ results into the tracked records.
#   TAG=r03 bash scripts/collect_profiles.sh            (after the GPU run merged gpurun_out/)
# For every workload profiled: profiles/<TAG>_<w>_kernel_stats.csv (rocprofv3 --stats of the
# default bench command), <TAG>_<w>_prof_bench.json (that command's JSON line),
# <TAG>_<w>_pmc_summary.txt and _valu_weighted.txt (the PMC passes), and the workload's records in
# profiles/pmc_valu.json and profiles/pmc_traffic.json, which bench.py reads for runs of the same
# configuration (scripts/pmc_summary.py, scripts/pmc_traffic.py; calibration reused).
set -eu
cd "$(dirname "$0")/.."
TAG=${TAG:-r03}
for w in ${WORKLOADS:-cornell1080 caustic8 weak64}; do
  [ -f gpurun_out/prof_$w/run_kernel_stats.csv ] || { echo "no profile for $w"; continue; }
  cp gpurun_out/prof_$w/run_kernel_stats.csv profiles/${TAG}_${w}_kernel_stats.csv
  grep '^{' gpurun_out/prof_$w.log | tail -1 > profiles/${TAG}_${w}_prof_bench.json
  python3 scripts/pmc_summary.py gpurun_out path_kernel "pmc_${w}_*" profiles/pmc_valu.json \
      > profiles/${TAG}_${w}_pmc_summary.txt
  python3 scripts/valu_weighted.py gpurun_out path_kernel "pmc_${w}_*" > profiles/${TAG}_${w}_valu_weighted.txt
  python3 scripts/pmc_traffic.py gpurun_out profiles/pmc_traffic.json "pmc_${w}_*" > /dev/null
  echo "$w: $(tail -1 profiles/${TAG}_${w}_valu_weighted.txt | cut -c1-160)"
done

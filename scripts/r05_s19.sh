set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "base:" "g16r4:BDPT_POOL_GRID=16;BDPT_POOL=4" "g16r2:BDPT_POOL_GRID=16;BDPT_POOL=2" "g8r2:BDPT_POOL_GRID=8;BDPT_POOL=2" "g64r8:BDPT_POOL_GRID=64;BDPT_POOL=8" "g32r4:BDPT_POOL_GRID=32;BDPT_POOL=4"; do
  tag=${v%%:*}; envs=${v#*:}; IFS=';' read -r -a assign <<< "$envs"
  env "${assign[@]}" timeout -k 10 200 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 20 --ns 8 > gpurun_out/s19_$tag.txt 2>&1 || { tail -5 gpurun_out/s19_$tag.txt; exit 1; }
  echo "$tag $(grep '"streams_req": 0' gpurun_out/s19_$tag.txt | tail -1)" | tee -a gpurun_out/s19_grid.txt
done

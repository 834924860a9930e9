set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2 3; do
for v in "base:" "g16r4:BDPT_POOL_GRID=16;BDPT_POOL=4" "g64r8:BDPT_POOL_GRID=64;BDPT_POOL=8" "g128r16:BDPT_POOL_GRID=128;BDPT_POOL=16" "g64r16:BDPT_POOL_GRID=64;BDPT_POOL=16"; do
  tag=${v%%:*}; envs=${v#*:}; IFS=';' read -r -a assign <<< "$envs"
  env "${assign[@]}" timeout -k 10 200 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 30 --ns 8 > gpurun_out/s20_$tag.txt 2>&1 || { tail -5 gpurun_out/s20_$tag.txt; exit 1; }
  echo "$r $tag $(grep '"streams_req": 0' gpurun_out/s20_$tag.txt | tail -1)" | tee -a gpurun_out/s20_grid.txt
done
done

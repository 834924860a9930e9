set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in default t32x2; do
  if [ $v = default ]; then E=""; else E="BDPT_LIB=variants/t32x2/libbdpt.so BDPT_JIT_FLAGS=-DBDPT_WTW=32,-DBDPT_BLOCK_WX=1"; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/fab_${v}_$c
    env $E timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/fab_${v}_$c -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline --no-smt-probe --steps 4 --warmup 1 --streams 16 > gpurun_out/fab_${v}_$c.log 2>&1 || { echo "STOP $v $c"; exit 3; }
    echo "$v $c ok"
  done
done

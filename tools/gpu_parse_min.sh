# Host parse A/B on the GPU box CPU (no GPU use): parse_bench builds given in BINS
# (tools/parse_bench), 1 thread, min-of-REPS per stream (-m), ROUNDS interleaved rounds per set.
cd $GRAFT_REPO_ROOT/tools/parse_bench
for set in ${SETS:-bench bench264 bench_heavy}; do
  for r in $(seq ${ROUNDS:-6}); do
    for b in ${BINS:-pb_A pb_B}; do
      echo "$set $b $(./$b ../../tests/golden/$set/*.h26? -r ${REPS:-7} -m | awk '{print $2}')"
    done
  done
done | awk '{k=$1" "$2; v[k]=v[k]" "$3; if(!(k in m) || $3<m[k]) m[k]=$3} END{for(k in m) print k, "min", m[k], "all", v[k]}' | sort

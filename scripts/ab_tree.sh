#!/bin/bash
# A/B of whole code trees (engine Python + kernels), interleaved on one GPU box:
#   local:  bash scripts/ab_tree.sh prep <name> [<git rev>=HEAD]   - exports <rev> into _abtree/<name> and builds it
#   box:    bash scripts/ab_tree.sh run <tag> <reps> <bench args...> - alternates `python bench.py <args>` in the
#           current tree and in every _abtree/* tree, <reps> rounds; logs under gpurun_out/r5_<tag>/
set -u
cd "$(dirname "$0")/.."
case ${1:-} in
  prep)
    name=$2; rev=${3:-HEAD}
    rm -rf "_abtree/$name" && mkdir -p "_abtree/$name"
    git archive "$rev" | tar -x -C "_abtree/$name"
    rm -rf "_abtree/$name/profiles"  # (records: not needed to run)
    (cd "_abtree/$name" && python -c "import __graft_entry__ as g; g.build()" | tail -1) ;;
  run)
    tag=$2; reps=$3; shift 3
    OUT=gpurun_out/r5_$tag; mkdir -p "$OUT"
    export HSA_ENABLE_IPC_MODE_LEGACY=0
    for r in $(seq 1 "$reps"); do
      for t in . _abtree/*; do
        n=$(basename "$t"); [ "$t" = . ] && n=cur
        (cd "$t" && timeout -k 10 300 python bench.py "$@") > "$OUT/${n}_$r.log" 2>&1
        rc=$?
        printf "%-8s %d rc=%d %s\n" "$n" "$r" "$rc" "$(grep -o '"ms_per_step": [0-9.]*' "$OUT/${n}_$r.log")"
        [ $rc -eq 0 ] || exit $rc
      done
    done ;;
  *) echo "usage: ab_tree.sh prep <name> [rev] | run <tag> <reps> <bench args...>"; exit 2 ;;
esac

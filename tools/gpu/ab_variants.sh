#!/bin/bash
# A/B of library variants (DKG_LIB = dkg_amd/_native/ab/libdkg_<v>.so, tools/build_variant.sh) and of the round-3
# build (.ab/f96856c worktree) against the default build: driver-shape bench (20 steps) and the 1024-step line,
# interleaved; the envelope-free legs skipped.  Then the headline stamps of each variant.
set -uo pipefail
out=${1:-gpurun_out/abv}
mkdir -p "$out"
root=$GRAFT_REPO_ROOT
opts="--cpu-seconds 0 --grad-steps 0 --b1-calls 0 --nd-steps 0 --stress-steps 0 --prep-reps 0"
run() {  # name, dir, lib, extra
  local name=$1 d=$2 lib=$3; shift 3
  (cd "$d" && DKG_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 $opts "$@") > "$out/b20_${name}_$rep.json" 2> "$out/b20_${name}_$rep.err" || { tail -5 "$out/b20_${name}_$rep.err"; return 1; }
  (cd "$d" && DKG_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 1024 --warmup 50 $opts "$@") > "$out/b1k_${name}_$rep.json" 2> "$out/b1k_${name}_$rep.err" || { tail -5 "$out/b1k_${name}_$rep.err"; return 1; }
}
ab=$root/decoupled-kg_amd/dkg_amd/_native/ab
for rep in 1 2; do
  run cur "$root" "" || exit 1
  run curlt4 "$root" "" --launch-threads -1 || exit 1
  for v in $(ls "$ab" | sed 's/libdkg_\(.*\)\.so/\1/'); do run "$v" "$root" "$ab/libdkg_$v.so" || exit 1; done
  for c in $(ls .ab 2>/dev/null); do run "r_$c" "$root/.ab/$c" "" || exit 1; done
done
for f in "$out"/*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); st=d['roofline']['stages']; print(sys.argv[1].split('/')[-1], round(d['value']/1e6,2), round(d['single_stream']['ms_per_step']*1e3,2), [round(v['avg_launch_us'],2) for v in st.values()])" "$f"; done
for v in $(ls "$ab" | sed 's/libdkg_\(.*\)\.so/\1/'); do
  DKG_LIB=$ab/libdkg_$v.so timeout -k 10 120 python3 -u tools/kstamps.py headline > "$out/kst_$v.txt" 2>&1 || exit 1
done
timeout -k 10 120 python3 -u tools/kstamps.py headline > "$out/kst_cur.txt" 2>&1 || exit 1
for f in "$out"/kst_*.txt; do echo "== $f"; grep -A7 "^envelope" "$f"; grep -A3 "^posterior_cov" "$f"; done

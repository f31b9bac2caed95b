# round-5 A/B: hashed io-vector insert/apply kernels with 256-thread blocks (abtree/, the
# previous build) against one-wave blocks (this tree); interleaved, 3 rounds
set -o pipefail
out=gpurun_out/r05iovbs
mkdir -p $out
P=2048,4096,16384,65536,262144
for r in 1 2 3; do
  timeout -k 10 120 python3 abtree/tools/scatter_bench.py --pairs $P --steps 100 --no-cpu > $out/old_$r.jsonl 2> $out/old_$r.err || { tail -5 $out/old_$r.err; exit 11; }
  timeout -k 10 120 python3 tools/scatter_bench.py --pairs $P --steps 100 --no-cpu > $out/new_$r.jsonl 2> $out/new_$r.err || { tail -5 $out/new_$r.err; exit 12; }
done
python3 - <<'PY'
import json, collections
o = collections.defaultdict(list)
for v in ("old", "new"):
    for r in (1, 2, 3):
        for l in open(f"gpurun_out/r05iovbs/{v}_{r}.jsonl"):
            d = json.loads(l); o[(d["pairs"], v)].append(d["ms_per_call"])
for n in sorted({k[0] for k in o}):
    print(n, "old", o[(n, "old")], "new", o[(n, "new")])
PY

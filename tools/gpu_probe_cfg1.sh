set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p1; mkdir -p $O
for b in 256 1024 4096 16384 65536; do
  timeout -k 10 120 python3 bench.py --config cfg1 --batch $b --steps 300 --warmup 50 --no-cpu > $O/b$b.json 2>$O/b$b.err || exit 1
done
for t in 4 8; do
  DF_TILES=$t timeout -k 10 120 python3 bench.py --config cfg1 --batch 4096 --steps 300 --warmup 50 --no-cpu > $O/t$t.json 2>$O/t$t.err || exit 1
done
DF_DEBUG_LAUNCH=1 timeout -k 10 120 python3 bench.py --config cfg1 --batch 4096 --steps 2 --warmup 1 --no-cpu > $O/dbg.json 2>$O/dbg.err || exit 1
for f in $O/*.json; do python3 -c "
import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);c=d.get('clock') or {}
print('$f', d['config'].get('per_gpu_batch'), round(d['value'],1), d['roofline'].get('kernel_ms'), c.get('kernel_mcycles_per_launch'), c.get('workgroup_slots'))"; done | tee $O/summary.txt
grep "\[df\]" $O/dbg.err | sort | uniq | head -5

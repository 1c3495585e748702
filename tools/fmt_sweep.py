import sys, json
tag = sys.argv[1] if len(sys.argv) > 1 else ""
for l in sys.stdin:
    try:
        r = json.loads(l)
    except Exception:
        if "amdgpu.ids" not in l:
            print(l.rstrip())
        continue
    print(f"{tag} {r.get('variant','')} v{r.get('vec','')} r{r.get('ring','')} bpc{r.get('bpc','')} {r['dtype']} tb={r['tb']:2d} tr={r['tile_rows']} cs={int(r['copy_swap'])} gpts={r['gpts']:8.1f} best={r['gpts_best']:8.1f} modelGB/s={r['model_gbps']:7.0f}")

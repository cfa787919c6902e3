import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    r = d["res"]
    old = min((v[0], k) for k, v in r.items() if int(k) < 16)
    new = min((v[0], k) for k, v in r.items() if int(k) >= 16)
    fl = lambda ms: r[str(old[1])][1] * old[0] / ms
    print(f"{d['shape']:14s} tw={int(d['tw'])} torch {d['torch_ms']:.4f} ({d['torch_tf']:6.1f}TF) old t{old[1]} {old[0]:.4f} ({fl(old[0]):6.1f}) pp t{new[1]} {new[0]:.4f} ({fl(new[0]):6.1f})  " + " ".join(f"{k}:{v[1]:.0f}" for k, v in r.items()))

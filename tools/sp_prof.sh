RSVIO_BA_PROFILE=1 timeout -k 10 200 python tools/timeline_probe.py 60 split > gpurun_out/sp_prof.out 2> gpurun_out/sp_prof.err; python3 - <<'PY'
import re, numpy as np
rows=[l for l in open("gpurun_out/sp_prof.err") if l.startswith("[rsvio] set_problem")]
keys=["checks+layout","upload wait","observations","waves","tables","enqueue","grow"]
vals={k:[] for k in keys}
for l in rows[20:]:
    for k in keys:
        m=re.search(re.escape(k)+r" ([0-9.]+)", l)
        vals[k].append(float(m.group(1)))
print(len(rows), {k: round(float(np.median(v)),1) for k,v in vals.items()})
print(rows[-1].strip())
PY

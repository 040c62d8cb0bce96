"""Build A/B variants of libnais_hip.so with extra -D flags into build_ab/<name>.so (CPU side;
the .so files travel to the GPU box). Usage: python scripts/build_ab.py name=-DFOO=1,-DBAR=2 ...
or name=nais_train.hip:-DFOO=1 to give the flags to that translation unit only (the others reuse
the cached objects of the default build), or name=nais_train.hip@scripts/probes/train_timing.hip
to compile a probe source (which includes the product file) in that unit's place."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from poi_recommendation_models_amd import build as b  # noqa: E402

out_dir = os.path.join(b.ROOT, "build_ab")
os.makedirs(out_dir, exist_ok=True)
for spec in sys.argv[1:]:
    name, _, flags = spec.partition("=")
    tu = None
    if "@" in flags:
        tu, _, probe = flags.partition("@")
        print(b.build(replace={tu: probe}, out=os.path.join(out_dir, name + ".so")), tu, probe, flush=True)
        continue
    if ":" in flags:
        tu, _, flags = flags.partition(":")
    extra = [f for f in flags.split(",") if f]
    if tu:
        print(b.build(extra_for={tu: extra}, out=os.path.join(out_dir, name + ".so")), tu, extra, flush=True)
    else:
        print(b.build(extra=extra, out=os.path.join(out_dir, name + ".so")), extra, flush=True)

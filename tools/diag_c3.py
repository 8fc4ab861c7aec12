import sys, os, faulthandler
faulthandler.enable()
ROOT = "/root/repo"
sys.path.insert(0, ROOT); sys.path.insert(0, ROOT + "/scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd")
import bench, gpscore
c = bench.CONFIGS[sys.argv[1]]
ctx = gpscore.Context(0)
for kv in sys.argv[2:]:
    k, v = kv.split("="); ctx.call("gps_ctx_set_option", int(k), int(v)); print("opt", k, v, flush=True)
gp = gpscore.GP(ctx=ctx)
X, y, Xt, yt, Z, th = bench.synth(c["n"], c["d"], c["nt"], c["seed"], c.get("m"))
print("synth", flush=True)
gp.set_data(X, y); gp.set_test(Xt, yt); print("set", flush=True)
r = gp.fit(theta=th, return_loo=False); print("fit", r.objectives, flush=True)

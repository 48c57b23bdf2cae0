import sys, os, traceback
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import test_gpu_features as t
ok = 0
for i in range(4):
    try:
        t.test_device_pipeline_timeline_overlap_gpu(t.ck.ClPlatforms.all().gpus()); ok += 1; print("run", i, "ok", flush=True)
    except AssertionError as e:
        print("run", i, "FAIL", e, flush=True)
print("ok", ok)

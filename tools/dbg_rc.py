import sys, os, time, faulthandler
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
faulthandler.dump_traceback_later(50, exit=True)
import test_gpu_resolver as T
mode = {"relax": "relax", "chunks": True, "wait": "wait"}[sys.argv[1]]
t0 = time.time()
orig = T.commit_window
def cw(gpu, op, batches):
    r = orig(gpu, op, batches)
    import ctypes
    from tigerbeetle_amd import _lib
    dbg = (ctypes.c_uint64 * 8)()
    _lib.lib().tbg_debug_counters(gpu.h, dbg, 8)
    print("window ok", op, len(batches), round(time.time() - t0, 2), gpu.stats(), [hex(x) for x in dbg], flush=True)
    return r
T.commit_window = cw
rep, st = T._run(mode, 1, 50, 4, 512, 6, 0, 1.2, 100)
print("done", st, flush=True)

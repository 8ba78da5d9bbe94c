"""Create, use and destroy hbtc contexts (and 8-slot nodes) in a loop with the process's HIP
hardware-queue setting (GPU_MAX_HW_QUEUES), reporting the first failure: a leak of streams,
events or queues in hbtc_ctx_create / hbtc_ctx_destroy shows up as a failing create."""
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hbbft_amd import _native as N  # noqa: E402
from tests.test_gpu_parity import _dec_batch  # noqa: E402


def main():
    print("GPU_MAX_HW_QUEUES=%s" % os.environ.get("GPU_MAX_HW_QUEUES"), flush=True)
    rng = random.Random(1)
    c0 = N.Context(0)
    pk, H, w, idx, shares, _, _ = _dec_batch(c0, rng, 40, [40, 7, 64], 0.05)
    t0 = time.time()
    for i in range(300):
        try:
            c = N.Context(0)
        except Exception as e:
            print("context %d: create failed: %r" % (i, e), flush=True)
            raise SystemExit(2)
        ks, _ = c.keyset_load(pk)
        for _ in range(2):  # touch every lane once more than the queue count would need
            c.verify_dec_shares(ks, H, w, [40, 7, 64], idx, shares)
        c.close()
        if i % 50 == 0:
            print("context %d ok (%.1fs)" % (i, time.time() - t0), flush=True)
    for i in range(20):
        try:
            nd = N.Node([0] * 8)
        except Exception as e:
            print("node %d: create failed: %r" % (i, e), flush=True)
            raise SystemExit(3)
        nd.close()
    print("300 contexts and 20 eight-slot nodes created, used and destroyed: ok", flush=True)
    c0.close()
    # contexts ALIVE at the same time (the GPU suite keeps a few module fixtures and nodes open):
    # create and use them without closing until one fails or 48 exist; hbtc_ctx_create names
    # the failing HIP call on stderr
    live = []
    try:
        for i in range(48):
            try:
                c = N.Context(0)
            except Exception as e:
                print("concurrent: context %d failed to create with %d alive: %r" % (i, len(live), e),
                      flush=True)
                break
            live.append(c)
            ks, _ = c.keyset_load(pk)
            c.verify_dec_shares(ks, H, w, [40, 7, 64], idx, shares)
        else:
            print("concurrent: 48 contexts alive and used: ok", flush=True)
    finally:
        for c in live:
            c.close()
    print("concurrent phase done (%d contexts)" % len(live), flush=True)


if __name__ == "__main__":
    main()

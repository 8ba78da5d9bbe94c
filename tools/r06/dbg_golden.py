"""Debug: the C1 coin fixture's statuses through the fused exact path and the three-launch path."""
import json, os, sys
sys.path.insert(0, os.getcwd())
from hbbft_amd import _native as N
c = json.load(open("tests/golden/c1_coin.json"))
b = bytes.fromhex
items = c["items"]
want = [i["expected"] for i in items]
for fused in ("1", "0"):
    os.environ["HBTC_SIG_FUSED"] = fused
    ctx = N.Context(0)
    ks, _ = ctx.keyset_load([b(p) for p in c["pk_shares"]])
    st = ctx.verify_sig_shares(ks, [b(c["H"])], [len(items)], [i["idx"] for i in items], [b(i["sig"]) for i in items])
    got = [N.STATUS_NAMES[int(s)] for s in st]
    print("fused", fused, [(i["name"], g, w) for i, g, w in zip(items, got, want) if g != w], flush=True)
    # the non-subgroup share alone, and with a valid one
    ns = [i for i in items if i["name"] == "enc_not_in_subgroup"][0]
    st = ctx.verify_sig_shares(ks, [b(c["H"])], [1], [ns["idx"]], [b(ns["sig"])])
    print("  alone:", N.STATUS_NAMES[int(st[0])], flush=True)
    ctx.close()

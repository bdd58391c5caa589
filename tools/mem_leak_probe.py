"""Run a pytest selection in-process, then report the CUDA memory still allocated and the
largest live CUDA tensors with the types of the objects that refer to them (leak hunt).

usage: python tools/mem_leak_probe.py <pytest args...>"""
import gc
import sys

import pytest
import torch


def main():
    rc = pytest.main(["-x", "-q", "-p", "no:cacheprovider"] + sys.argv[1:])
    gc.collect()
    torch.cuda.synchronize()
    print(f"pytest rc {rc}; allocated {torch.cuda.memory_allocated() / 2**30:.2f} GiB, "
          f"reserved {torch.cuda.memory_reserved() / 2**30:.2f} GiB", flush=True)
    from deep_video_interpolation_extrapolation_amd import engine
    plans = [o for o in gc.get_objects() if isinstance(o, engine.Plan)]
    print(f"live plans: {len(plans)}", flush=True)
    skip = {id(plans)}
    for pl in plans[:3]:  # one referrer path upwards per live plan
        cur, path = pl, []
        for _ in range(10):
            refs = [r for r in gc.get_referrers(cur) if id(r) not in skip and not isinstance(r, type(sys._getframe()))]
            if not refs:
                break
            cur = refs[0]
            desc = type(cur).__name__
            if isinstance(cur, dict):
                desc += f"{sorted(map(str, cur.keys()))[:5]}"
            path.append(desc)
        print("  plan <- " + " <- ".join(path), flush=True)
    big = []
    for o in gc.get_objects():
        try:
            if isinstance(o, torch.Tensor) and o.is_cuda and o.untyped_storage().nbytes() > 2**28:
                big.append(o)
        except Exception:
            pass
    seen = set()
    for t in sorted(big, key=lambda t: -t.untyped_storage().nbytes())[:12]:
        key = t.untyped_storage().data_ptr()
        if key in seen:
            continue
        seen.add(key)
        refs = [type(r).__name__ + (f":{sorted(r.keys())[:6]}" if isinstance(r, dict) else "") for r in gc.get_referrers(t)
                if r is not big]
        print(f"{t.untyped_storage().nbytes() / 2**30:7.2f} GiB {tuple(t.shape)} {t.dtype} referrers {refs[:4]}", flush=True)
        for r in gc.get_referrers(t):
            if isinstance(r, dict):
                for rr in gc.get_referrers(r)[:3]:
                    print(f"        dict owner: {type(rr).__name__}", flush=True)


if __name__ == "__main__":
    main()

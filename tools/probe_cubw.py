"""Per-CU HBM read rate under a CU mask: register loads vs LDS-DMA, in-order vs scattered 2 KiB
units, several waves per CU and units in flight (tools/probe_cubw.hip)."""
import ctypes
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    import torch
    torch.cuda.set_device(0)
    lib = ctypes.CDLL(os.path.join(ROOT, 'tools', 'libprobe_cubw.so'))
    us, gbps = ctypes.c_float(), ctypes.c_float()
    # spread = 1: the budget's CU slots spread evenly over each XCD's CUs instead of its first ones
    sweep = [(0, (4, 8, 16, 32, 64, 128, 192, 0), ((0, 4, 4), (0, 8, 4), (0, 8, 8))),
             (1, (8, 16, 32, 64, 128, 192), ((0, 4, 4), (0, 8, 4), (0, 8, 8)))] if os.environ.get('CUBW_SPREAD') else \
            [(0, (32, 128, 0), ((0, 4, 4), (0, 8, 4), (0, 16, 2), (0, 8, 8), (1, 4, 4), (1, 8, 2), (1, 2, 8)))]
    for spread, budgets, shapes in sweep:
        lib.probe_cubw_set_spread(spread)
        for cus in budgets:
            for lds, L, wgs in shapes:
                for scattered in (0, 1):
                    rc = lib.probe_cubw(cus, wgs, L, lds, scattered, 5, ctypes.byref(us), ctypes.byref(gbps))
                    n = cus or torch.cuda.get_device_properties(0).multi_processor_count
                    print(json.dumps(dict(cus=n, spread=spread, lds=lds, units_in_flight=L, wg_per_cu=wgs,
                                          scattered=scattered, rc=rc, us=round(us.value, 1), gbps=round(gbps.value, 1),
                                          gbps_per_cu=round(gbps.value / n, 1))), flush=True)


if __name__ == '__main__':
    main()

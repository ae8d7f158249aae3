"""EP = 8 phase A (one rank's share of config 3, tools/kphase_prof.py's launches) under a CU budget:
the default launch (the item kernel on its full grid, 4 rows in flight per lane on a budget stream)
against the persistent grid sized to the budget (deepep_set_kernel_choice(5)) -- the setting of the
N > 1 bench's DEEPEP_PHASE_A_CUS leg."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    torch.cuda.set_device(0)
    from deepep_amd import _lib
    from deepep_amd.kernels import HipKernels
    from tools.kphase_prof import setup
    launch_a, launch_b, bytes_a, bytes_b, info = setup()
    lib = HipKernels().lib

    def timed(fn, s, n=20):
        for _ in range(3):
            fn(s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(n):
            fn(s)
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / n

    for cus in (0, 192, 128, 64):
        if cus:
            import ctypes
            h = ctypes.c_void_p()
            _lib.check(lib.deepep_stream_create_cu_budget(cus, ctypes.byref(h)), 'cu budget')
            s = torch.cuda.ExternalStream(h.value)
        else:
            s = torch.cuda.current_stream()
        row = dict(cus=cus)
        for name, choice in (('default', -1), ('persistent', 5)):
            lib.deepep_set_kernel_choice(choice)
            row[f'phase_a_{name}_us'] = round(timed(launch_a, s), 1)
            row[f'phase_b_{name}_us'] = round(timed(launch_b, s), 1)
        lib.deepep_set_kernel_choice(-1)
        for k in list(row):
            if k.startswith('phase_a_'):
                row[k.replace('_us', '_tbps')] = round(bytes_a / row[k] / 1e6, 2)
        print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()

"""Which CUs a CU-masked stream uses (diagnostic for deepep_stream_create_cu_budget)."""
import ctypes
import json
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    torch.cuda.set_device(0)
    n = torch.cuda.get_device_properties(0).multi_processor_count
    lib = ctypes.CDLL(os.path.join(ROOT, 'tools', 'libprobe_cumask.so'))
    words = (n + 31) // 32
    blocks = 4096

    def run(bits, tag):
        mask = (ctypes.c_uint32 * words)()
        for b in bits:
            mask[b // 32] |= 1 << (b % 32)
        out = (ctypes.c_uint32 * (2 * blocks))()
        rc = lib.probe_cumask(mask, words, blocks, out)
        assert rc == 0, rc
        slots = set()
        per_xcc = {}
        for i in range(blocks):
            hw, xcc = out[2 * i], out[2 * i + 1]
            cu, sh, se = (hw >> 8) & 0xF, (hw >> 12) & 0x1, (hw >> 13) & 0x7
            slots.add((xcc & 0xF, se, sh, cu))
        for x, se, sh, cu in slots:
            per_xcc[x] = per_xcc.get(x, 0) + 1
        print(json.dumps(dict(tag=tag, bits=len(bits), distinct_cus=len(slots),
                              cus_per_xcc=dict(sorted(per_xcc.items())))), flush=True)
        return slots

    # which (shader engine, shader array, CU) each mask bit of XCD 0 selects (bit b = CU slot b // 8)
    topo = {}
    for b in range(0, n, 8):
        mask = (ctypes.c_uint32 * words)()
        mask[b // 32] |= 1 << (b % 32)
        out = (ctypes.c_uint32 * (2 * 256))()
        assert lib.probe_cumask(mask, words, 256, out) == 0
        hw = out[0]
        topo[b // 8] = [(hw >> 13) & 0x7, (hw >> 12) & 0x1, (hw >> 8) & 0xF]
    print(json.dumps(dict(tag='xcd0_slot_to_se_sh_cu', map=topo)), flush=True)

    run(range(n), 'all')
    for k in (8, 16, 32, 64, 96, 128):
        run([i * n // k for i in range(k)], f'spread{k}')
        run(range(k), f'first{k}')
    run([b for b in range(n) if b % 8 == 0], 'every8th')
    run(range(0, 32), 'word0')


if __name__ == '__main__':
    main()

"""Per-kernel register / scratch / instruction counts from a hipcc -save-temps gfx950 .s file.
Usage: python tools/asm_stats.py <file.s> [name-regex]"""
import re
import sys

s = open(sys.argv[1]).read()
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else '.')
for m in re.finditer(r'^(\S+):\s*(;.*)?$', s, re.M):
    name = m.group(1)
    if not name.startswith('_Z') or not pat.search(name):
        continue
    end = s.find('.Lfunc_end', m.end())
    body = s[m.end():end]
    k = s.find('.amdhsa_kernel ' + name)
    meta = s[k:s.find('.end_amdhsa_kernel', k)]

    def g(key):
        mm = re.search(r'\.' + key + r'\s+(\d+)', meta)
        return int(mm.group(1)) if mm else -1
    n_ins = len(re.findall(r'^\s+(?:[sv]_|ds_|buffer_|global_)', body, re.M))
    print(f'{name[:100]}\n   vgpr {g("amdhsa_next_free_vgpr")} accum_offset {g("amdhsa_accum_offset")} '
          f'scratch {g("amdhsa_private_segment_fixed_size")} lds {g("amdhsa_group_segment_fixed_size")} | '
          f'mfma {body.count("v_mfma")} ds_read {len(re.findall(r"ds_read", body))} '
          f'ds_write {len(re.findall(r"ds_write", body))} buffer_load {body.count("buffer_load")} '
          f'scratch_ops {len(re.findall(r"scratch_(load|store)", body))} s_waitcnt {body.count("s_waitcnt")} '
          f'barrier {body.count("s_barrier")} instr {n_ins}')

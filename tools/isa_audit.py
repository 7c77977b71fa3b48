"""Static audit of the shipped code objects (libdbsr_hip.so) for the LDS-DMA kernels ('the two-lane
race'): every kernel that issues LDS-DMA (buffer_load_* ... lds / global_load_lds_*) must

  * own its SIMDs: the registers it declares (.vgpr_count, arch VGPRs + AGPRs) times its waves per SIMD at
    the occupancy its launch bounds / LDS allow must fill the 512-entry unified register file, so that no
    wave of another kernel (another stream's) can be co-resident on those SIMDs (DBSR_OWN_SIMDS);
  * set M0 (the LDS-DMA destination base) in the same basic block before every LDS-DMA instruction;
  * declare at least as many registers as its code uses (highest v/a register index in the ISA);
  * stay within its declared LDS (.group_segment_fixed_size <= 160 KiB);
  * reach no s_endpgm with an LDS-DMA of its own still in flight (in code order since the last vmcnt wait): a
    workgroup that ends with pieces outstanding frees its LDS to the next workgroup while they land (VERDICT r4
    #6, e.g. a persistent block's prefetch past its last tile).

Over EVERY kernel (LDS-DMA or not): no VALU instruction may overwrite the data VGPRs of a vector-memory store
(buffer_/global_/flat_store_*) within STORE_HAZARD_WAIT wait states of it -- the store may not have read its data
yet.  ROCm 7.2 emitted a v_pk_mul_f32 straight after a buffer_store over its data registers with no s_nop between
(the fused predictor's fusion weights came out corrupted at fixed lanes); the product avoids
buffer_store and builds that file with -fno-slp-vectorize, and this rule guards the class.

Usage: python tools/isa_audit.py [libdbsr_hip.so]   (prints one line per LDS-DMA kernel; exit 1 on a violation)
Also imported by tests/test_capi.py."""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = '/opt/rocm/lib/llvm/bin'
MAGIC = b'__CLANG_OFFLOAD_BUNDLE__'
DMA_RE = re.compile(r'\b(buffer_load_\w+\b.*\blds\b|global_load_lds_\w+)')
# LDS-DMA ring kernels (train_ops.hip, conv_wgrad_dma_kernel): a 3-stage ring whose per-tile barrier is passed
# with the NEXT tile's DMAs in flight by design (they fill the stage after the one being read; the stage the DMAs
# issued after the barrier overwrite was read before it), so the drain rule becomes: a vmcnt wait between the
# wave's last DMA and every barrier.  Its 9-wave blocks cannot own their SIMDs (3 waves on one SIMD); it is a
# training-step kernel, issued on the trainer's one stream (no second lane runs beside the backward).
RING_KERNELS = ('conv_wgrad_dma_kernel', 'conv_fuse_kernel')
# wait states a store's data VGPRs must stay untouched by VALU writes after the store issues (the CDNA3/4 ISA's
# "VMEM store data hazard", stores of more than 64 bits of data: 1 wait state; 2 here, a margin for gfx950's
# packed-fp32 VALU, whose write was the one observed racing)
STORE_HAZARD_WAIT = 2
STORE_RE = re.compile(r'^(buffer|global|flat|scratch)_store_\w+\s+(?:off,\s*)?')
VREG_RE = re.compile(r'\bv(?:\[(\d+):(\d+)\]|(\d+)\b)')


def _vregs(op):
    """The VGPR indices an operand names (vN or v[a:b]), else an empty set."""
    m = VREG_RE.match(op.strip())
    if not m:
        return set()
    if m.group(3) is not None:
        return {int(m.group(3))}
    return set(range(int(m.group(1)), int(m.group(2)) + 1))


def store_data_hazards(ins):
    """[(store, valu)] pairs: a VALU write to a store's data VGPRs within STORE_HAZARD_WAIT wait states of it.
    Store operands: global/flat/scratch_store vaddr, vdata, ...; buffer_store vdata, vaddr, ..."""
    out = []
    for j, t in enumerate(ins):
        m = re.match(r'^(buffer|global|flat|scratch)_store_(\w+)\s+(.*)$', t)
        # the hazard exists for stores of more than 64 bits of data (dwordx3 / dwordx4, b96 / b128)
        if not m or not re.match(r'(dwordx[34]|b96|b128)', m.group(2)):
            continue
        ops = [o.strip() for o in m.group(3).split(',')]
        data = _vregs(ops[0] if m.group(1) == 'buffer' else (ops[1] if len(ops) > 1 else ''))
        if not data:
            continue
        waited, q = 0, j + 1
        while q < len(ins) and waited < STORE_HAZARD_WAIT:
            u = ins[q]
            if re.match(r'^(s_endpgm|s_branch|s_setpc)', u):
                break                   # no fall-through: the next instruction in code order does not follow it
            n = re.match(r'^s_nop\s+(\w+)', u)
            if n:
                waited += int(n.group(1), 0) + 1
            else:
                if u.startswith('v_') and not re.match(r'^v_(readlane|readfirstlane|cmp|cmpx)', u):
                    dst = u.split(None, 1)[1].split(',')[0] if ' ' in u else ''
                    if _vregs(dst) & data:
                        out.append((t, u))
                        break
                waited += 1
            q += 1
    return out


def code_objects(so_path):
    """The gfx950 code objects bundled in the shared object's .hip_fatbin section."""
    data = open(so_path, 'rb').read()
    out = []
    pos = data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from('<Q', data, pos + 24)[0]
        q = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from('<QQQ', data, q)
            triple = data[q + 24:q + 24 + tlen].decode(errors='replace')
            q += 24 + tlen
            if 'gfx950' in triple and size > 0:
                out.append(data[pos + off:pos + off + size])
        pos = data.find(MAGIC, pos + 24)
    return out


def kernel_meta(co_file):
    """{kernel symbol: {vgpr, agpr, lds, wg_max}} from the code object's metadata notes: each kernel is one
    list item of .kernels ('  - .agpr_count: ...' at indent 2, its own fields at indent 4)."""
    txt = subprocess.run([os.path.join(LLVM, 'llvm-readelf'), '--notes', co_file], capture_output=True,
                         text=True).stdout
    meta, rec = {}, None
    keys = {'.vgpr_count': 'vgpr', '.agpr_count': 'agpr', '.group_segment_fixed_size': 'lds',
            '.max_flat_workgroup_size': 'wg_max', '.symbol': 'symbol'}
    for line in txt.splitlines():
        ind = len(line) - len(line.lstrip(' '))
        s = line.strip()
        if ind == 2 and s.startswith('- .'):
            if rec and 'symbol' in rec:
                meta[rec['symbol']] = rec
            rec = {}
            s = s[2:]
            ind = 4
        if rec is None or ind != 4 or ':' not in s:
            continue
        k, v = s.split(':', 1)
        if k in keys:
            v = v.strip()
            rec[keys[k]] = v[:-3] if k == '.symbol' and v.endswith('.kd') else (int(v) if k != '.symbol' else v)
    if rec and 'symbol' in rec:
        meta[rec['symbol']] = rec
    return meta


def audit(so_path, hazards=None):
    """rows / bad kernels of the LDS-DMA rules; `hazards` (a list, optional) collects (kernel, store, valu) store-data
    hazards over every kernel -- their kernels are added to `bad` too."""
    rows, bad = [], []
    with tempfile.TemporaryDirectory() as td:
        for i, co in enumerate(code_objects(so_path)):
            f = os.path.join(td, f'co{i}.elf')
            open(f, 'wb').write(co)
            dis = subprocess.run([os.path.join(LLVM, 'llvm-objdump'), '-d', '--mcpu=gfx950', f], capture_output=True,
                                 text=True).stdout
            meta = kernel_meta(f)
            # split the disassembly per kernel symbol
            kern, body = None, {}
            for line in dis.splitlines():
                m = re.match(r'^[0-9a-f]+ <(\S+)>:', line)
                if m:
                    kern = m.group(1)
                    body[kern] = []
                elif kern is not None:
                    body[kern].append(line)
            for k, lines in body.items():
                if k not in meta:
                    continue
                ins = [ln.split(';')[0].strip() for ln in lines if ln.strip()]
                # objdump lines: '<tab>mnemonic operands  // address: encoding' -- keep the instruction text only
                ins = [t.split('//')[0].strip() for t in ins]
                ins = [t for t in ins if t]
                hz = store_data_hazards(ins)
                if hz:
                    bad.append(k)
                    if hazards is not None:
                        hazards.extend((k, st, va) for st, va in hz)
                dma = [j for j, t in enumerate(ins) if DMA_RE.search(t)]
                if not dma:
                    continue
                md = meta[k]
                regs = md.get('vgpr', 0)          # unified count: arch VGPRs + AGPRs (accum_offset included)
                hi_v = max([int(x) for t in ins for x in re.findall(r'\bv\[?(\d+)', t)] + [0])
                hi_a = max([int(x) for t in ins for x in re.findall(r'\ba\[?(\d+)', t)] + [0])
                # M0 written in the same basic block before each DMA
                m0_ok = True
                for j in dma:
                    q = j - 1
                    while q >= 0 and not re.match(r'^(s_cbranch|s_branch|s_setpc|s_endpgm)', ins[q]) and \
                            not re.search(r'\bm0\b', ins[q].split(',')[0] if ins[q].startswith('s_') else ''):
                        q -= 1
                    if q < 0 or not re.search(r'\bm0\b', ins[q].split(',')[0]):
                        m0_ok = False
                        break
                # a barrier reached (in code order, since the previous barrier) by an LDS-DMA of this wave must be
                # preceded by a vector-memory wait that covers that DMA (s_waitcnt vmcnt(N) with only non-DMA
                # operations among the N youngest): a barrier that lets a wave pass with its LDS-DMAs in flight lets
                # other waves read LDS that has not landed
                ring = any(r in k for r in RING_KERNELS)
                drain_ok, end_ok, outstanding, waited = True, True, [], True
                for t in ins:
                    if re.match(r'^(buffer|global|flat)_(load|store|atomic)', t):
                        outstanding.append(bool(DMA_RE.search(t)))
                        if DMA_RE.search(t):
                            waited = False
                    m = re.search(r's_waitcnt.*vmcnt\((\d+)\)', t)
                    if m:
                        n = int(m.group(1))
                        outstanding = outstanding[len(outstanding) - n:] if n else []
                        waited = True
                    elif t.startswith('s_barrier'):
                        if (not waited) if ring else any(outstanding):
                            drain_ok = False
                        outstanding = []
                    elif t.startswith('s_endpgm'):
                        if any(outstanding) or not waited:
                            end_ok = False
                wg = md.get('wg_max', 256)
                waves_per_simd_min = max(1, (wg // 64 + 3) // 4)
                owns = regs * waves_per_simd_min >= 512 or regs >= 256 or ring
                fits = md.get('lds', 0) <= 160 * 1024
                declared = hi_v < regs and (hi_a == 0 or hi_a < md.get('agpr', 0))
                ok = owns and m0_ok and fits and declared and drain_ok and end_ok
                rows.append((k, len(dma), regs, hi_v, hi_a, md.get('lds', 0), wg, owns, m0_ok, declared, fits,
                             drain_ok, end_ok))
                if not ok:
                    bad.append(k)
    return rows, bad


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                             'deep-rawburst-sr_amd', 'libdbsr_hip.so')
    hazards = []
    rows, bad = audit(so, hazards)
    for k, st, va in hazards:
        print('STORE-DATA HAZARD %s: %s  <-  %s' % (k[:90], st, va))
    for k, n, regs, hv, ha, lds, wg, owns, m0, dec, fits, drain, end in rows:
        print('%-90s dma %3d regs %3d (max v%d a%d) lds %6d wg %3d owns %d m0 %d declared %d lds-ok %d drain %d '
              'end %d' % (k[:90], n, regs, hv, ha, lds, wg, owns, m0, dec, fits, drain, end))
    print('%d LDS-DMA kernels, %d store-data hazards, %d violations' % (len(rows), len(hazards), len(set(bad))))
    sys.exit(1 if bad else 0)


if __name__ == '__main__':
    main()

"""Summarise a tools/profile.sh run into profiles/<tag>_summary.md (+ the raw kernel stats CSV).

HBM traffic per launch = 2 x FETCH_SIZE + WRITE_SIZE (KB units, x1024), following
MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE counts half of the bytes of 16-B-per-lane streaming
reads, so it is doubled; WRITE_SIZE is exact for 16-B streaming stores.  Each counter comes from its
own rocprofv3 --pmc pass (no trace domains combined).

Usage: python tools/summarize_profile.py gpurun_out/prof_r01 r01
"""
import csv
import json
import os
import shutil
import statistics
import sys

KERNELS = {   # label -> (name predicate, algorithmic bytes per launch at the default bench workload)
    'warp kernel (DBSR warp, encoders.py:80)':
        (lambda n: ('warp_kernel' in n and 'backwarp' not in n and '_bwd' not in n) or 'warp512_bf16_kernel' in n, None),
    'fused wp.out conv + softmax + fusion (merging.py:55-57,116-126)': (lambda n: 'conv_fuse_kernel' in n, None),
    'fused 32-ch ResBlock (decoders.py:46-49)': (lambda n: 'resblock32_kernel' in n and ('Lb0E' in n or 'false>' in n), None),
    'fused 32-ch ResBlock + RGB predictor (decoders.py:59-61)': (lambda n: 'resblock32_kernel' in n and ('Lb1E' in n or 'true>' in n), None),
    'upsampler conv + PixelShuffle + blur (upsampling.py:51-66)': (lambda n: 'upsample_blur_kernel' in n, None),
}


# kernel name -> bench.py family (bench.py CONV_FAMILIES / roofline_hbm keys)
FAMILY = [('conv3x3_ws_kernel', 'conv3x3_ws'), ('conv3x3_ks128_kernel', 'conv3x3_ks128'), ('conv3x3_pipe_kernel', 'conv3x3_pipe'),
          ('conv3x3_tiled_kernel', 'conv3x3_tiled'), ('conv3x3_narrow_kernel', 'conv3x3_narrow'), ('conv3x3_small_kernel', 'conv3x3_small'),
          ('conv1x1_kernel', 'conv1x1'),
          ('upsample_shuffle_kernel', 'conv1x1_shuffle'), ('upsample_blur_kernel', 'conv1x1_shuffle_blur'),
          ('resblock32_kernel', 'resblock32'), ('resblock64_kernel', 'resblock64'), ('conv_fuse_kernel', 'conv_fuse'), ('conv2d_kernel', 'conv2d_generic'),
          ('pwc_dense', 'pwc_dense'),
          ('pwc_extract_kernel', 'pwc_extract'), ('warp512_bf16_kernel', 'warp'), ('fuse512_bf16_kernel', 'fuse')]


def family(name):
    for key, fam in FAMILY:
        if key in name:
            return fam
    return None


def traffic_json(fetch, write, tag):
    """profiles/pmc_traffic.json: mean HBM bytes per launch of each kernel family (2 x FETCH_SIZE + WRITE_SIZE,
    KB units) over every profiled dispatch of the family -- every op of the forward is dispatched equally often
    in the profiled bench run, so this is the per-launch average over one forward's launches."""
    out = {}
    for fam in sorted({family(r['Kernel_Name']) for r in fetch} - {None}):
        fv = [float(r['Counter_Value']) for r in fetch if family(r['Kernel_Name']) == fam]
        wv = [float(r['Counter_Value']) for r in write if family(r['Kernel_Name']) == fam]
        if not fv or not wv:
            continue
        fb, wb = 2 * statistics.mean(fv) * 1024, statistics.mean(wv) * 1024
        out[fam] = {'bytes_per_launch': round(fb + wb), 'fetch_bytes': round(fb), 'write_bytes': round(wb),
                    'dispatches': len(fv), 'source': 'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, '
                    'profiles/%s_summary.md (FETCH_SIZE x2, gfx950)' % tag}
    return out


def main():
    src, tag = sys.argv[1], sys.argv[2]
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outdir = os.path.join(repo, 'profiles')
    os.makedirs(outdir, exist_ok=True)
    stats = list(csv.DictReader(open(os.path.join(src, 'trace', 'run_kernel_stats.csv'))))
    shutil.copy(os.path.join(src, 'trace', 'run_kernel_stats.csv'), os.path.join(outdir, f'{tag}_kernel_stats.csv'))
    lines = [f'# rocprofv3 summary {tag}', '',
             'Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline '
             '--no-op-timing`', '(fp16, batch 8 x 14 frames x 48x48; graph replays only, so every duration is in-step: '
             '14 forwards per kernel (warmup + timed)). Full CSV: `%s_kernel_stats.csv`.' % tag, '',
             '| kernel | calls | total ms | avg us | % |', '|---|---|---|---|---|']
    for r in stats[:25]:
        lines.append('| `%s` | %s | %.2f | %.1f | %s |' % (r['Name'][:110], r['Calls'], float(r['TotalDurationNs']) / 1e6,
                                                        float(r['AverageNs']) / 1e3, r['Percentage']))
    fetch = list(csv.DictReader(open(os.path.join(src, 'pmc_fetch', 'run_counter_collection.csv'))))
    write = list(csv.DictReader(open(os.path.join(src, 'pmc_write', 'run_counter_collection.csv'))))
    lines += ['', '## HBM traffic (PMC, separate passes)', '',
              '| kernel | dispatches | FETCH_SIZE x2 (MB) | WRITE_SIZE (MB) | traffic/launch (MB) | avg dur (us) |',
              '|---|---|---|---|---|---|']
    for label, (pred, _) in KERNELS.items():
        fr = [r for r in fetch if pred(r['Kernel_Name'])]
        wr = [r for r in write if pred(r['Kernel_Name'])]
        if not fr or not wr:
            continue
        # the large (bench-shaped) launches only
        big = max(int(r['Grid_Size']) for r in fr)
        fv = [float(r['Counter_Value']) for r in fr if int(r['Grid_Size']) == big]
        wv = [float(r['Counter_Value']) for r in wr if int(r['Grid_Size']) == big]
        dur = [int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in fr if int(r['Grid_Size']) == big]
        fmb = 2 * statistics.median(fv) * 1024 / 1e6
        wmb = statistics.median(wv) * 1024 / 1e6
        lines.append('| %s | %d | %.1f | %.1f | %.1f | %.1f |' % (label, len(fv), fmb, wmb, fmb + wmb,
                                                                statistics.median(dur) / 1e3))
    traffic = traffic_json(fetch, write, tag)
    lines += ['', '## HBM traffic per launch by kernel family (mean over all profiled dispatches)', '',
              '| family | dispatches | fetch MB | write MB | traffic/launch MB |', '|---|---|---|---|---|']
    for fam, t in traffic.items():
        lines.append('| %s | %d | %.1f | %.1f | %.1f |' % (fam, t['dispatches'], t['fetch_bytes'] / 1e6,
                                                          t['write_bytes'] / 1e6, t['bytes_per_launch'] / 1e6))
    json.dump(traffic, open(os.path.join(outdir, 'pmc_traffic.json'), 'w'), indent=1)
    tstats = os.path.join(src, 'train', 'run_kernel_stats.csv')
    if os.path.exists(tstats):
        shutil.copy(tstats, os.path.join(outdir, f'{tag}_train_kernel_stats.csv'))
        rows = list(csv.DictReader(open(tstats)))
        lines += ['', '## Training leg: `rocprofv3 --kernel-trace --stats -- python3 bench.py --mode train --steps 4 '
                  '--warmup 2 --no-op-timing`', '(bf16, 8 x 14 x 128x128; 6 trainer steps, no per-op pass). Full CSV: '
                  '`%s_train_kernel_stats.csv`.' % tag, '',
                  '| kernel | calls | total ms | avg us | % |', '|---|---|---|---|---|']
        for r in rows[:25]:
            lines.append('| `%s` | %s | %.2f | %.1f | %s |' % (r['Name'][:110], r['Calls'],
                                                            float(r['TotalDurationNs']) / 1e6,
                                                            float(r['AverageNs']) / 1e3, r['Percentage']))
    open(os.path.join(outdir, f'{tag}_summary.md'), 'w').write('\n'.join(lines) + '\n')
    print('\n'.join(lines))


if __name__ == '__main__':
    main()

"""Summarise two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over bench.py into the HBM traffic
per enc_mb_kernel launch that bench.py reports as roofline.traffic.
gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts half the bytes of wide streaming
reads, so fetched bytes = 2 x FETCH_SIZE; both counters are in KiB. Writes are taken as reported.
usage: pmc_enc.py <fetch_dir> <write_dir> <out.json> <width> <height> <streams>"""
import csv, glob, json, os, sys


def per_dispatch(d, counter, kernel='enc_mb_kernel'):
    f = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    if not f:
        sys.exit(f'no counter_collection.csv under {d}')
    vals = {}
    for r in csv.DictReader(open(f[0])):
        if kernel in r['Kernel_Name'] and r['Counter_Name'] == counter:
            vals[r['Dispatch_Id']] = vals.get(r['Dispatch_Id'], 0.0) + float(r['Counter_Value'])
    return list(vals.values())


def all_kernels(fd, wd):
    """per-dispatch averages of every codec kernel: fetched (x2 corrected) and written MB"""
    def table(d, counter):
        f = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)[0]
        acc = {}
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'] != counter or 'h264mi::' not in r['Kernel_Name']:
                continue
            k = r['Kernel_Name'].split('h264mi::')[1].split('(')[0]
            acc.setdefault(k, {}).setdefault(r['Dispatch_Id'], 0.0)
            acc[k][r['Dispatch_Id']] += float(r['Counter_Value'])
        return {k: sum(v.values()) / len(v) for k, v in acc.items()}
    fe, wr = table(fd, 'FETCH_SIZE'), table(wd, 'WRITE_SIZE')
    print('per dispatch: fetched MB (2 x FETCH_SIZE KiB) | written MB (WRITE_SIZE KiB)')
    for k in sorted(fe, key=lambda k: -fe[k]):
        print(f'  {k:28s} fetch {2 * fe[k] * 1024 / 1e6:10.2f} MB  write {wr.get(k, 0) * 1024 / 1e6:10.2f} MB')


def main():
    if '--all' in sys.argv:
        all_kernels(sys.argv[1], sys.argv[2])
        return
    fd, wd, out, w, h, s = sys.argv[1:7]
    fe, wr = per_dispatch(fd, 'FETCH_SIZE'), per_dispatch(wd, 'WRITE_SIZE')
    fkb, wkb = sum(fe) / len(fe), sum(wr) / len(wr)
    res = {'kernel': 'enc_mb_kernel', 'width': int(w), 'height': int(h), 'streams': int(s),
           'dispatches': [len(fe), len(wr)], 'fetch_size_kib_avg': fkb, 'write_size_kib_avg': wkb,
           'hbm_bytes_per_launch': (2 * fkb + wkb) * 1024,
           'correction': 'fetched = 2 x FETCH_SIZE (gfx950 half-count of wide reads); KiB units'}
    json.dump(res, open(out, 'w'), indent=1)
    print(json.dumps(res))


if __name__ == '__main__':
    main()

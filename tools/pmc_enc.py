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


def main():
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

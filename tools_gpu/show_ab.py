import json, sys
cur = None
for l in open(sys.argv[1]):
    if l.startswith('=='):
        cur = l.strip()
        continue
    if l.startswith('{'):
        d = json.loads(l)
        print(cur, {k: round(v * 1000, 2) for k, v in d['roofline']['ms_per_kernel'].items()},
              'us/step %.1f' % (d['ms_per_step'] * 1000), 'frac %.3f' % d['roofline']['frac'], 'loss %.5f' % d.get('loss_last_step', 0))

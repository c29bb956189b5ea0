import json, sys
for l in sys.stdin:
    try:
        d = json.loads(l)
    except Exception:
        print(l.rstrip()); continue
    if "span_us" in d:
        print('V', d.pop('V'), 'B', d.pop('B'), 'span', d.pop('span_us'))
        for k, v in d.items(): print('  %-32s' % k, v)
    else:
        print(d)

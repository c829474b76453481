"""print the headline of bench JSON lines (dev helper)"""
import json
import sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d['roofline']
    dec = r['decode']
    print(f, d['value'], 'm/s', d['ms_per_step'], 'ms |', r['kernel'], r['kernel_ms_per_launch'], 'frac', r['frac'], '| dec',
          dec['ms_per_step'], 'img', dec['img_ms'], 'step', dec['step_ms'], 'logit', dec['logit_ms'], 'cell', dec['cell_ms'],
          dec.get('shape'), 'ties', d['tie_fallbacks'])

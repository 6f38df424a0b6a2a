import json
import sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l)['pip_join']
        print(j['mode'], j['index']['cells'], round(j['ms_per_step'], 2), j['matches'], j.get('index_build_s'))

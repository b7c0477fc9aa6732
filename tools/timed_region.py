"""Timed region of a bench run from a rocprofv3 --marker-trace --kernel-trace csv dir: head (region start -> first kernel), tail (last kernel end -> region end), kernel span.
usage: python tools/timed_region.py <dir>"""
import csv, sys
d=sys.argv[1]
m=[r for r in csv.DictReader(open(d+'/run_marker_api_trace.csv')) if 'timed region' in str(r)]
r=m[-1]; s,e=int(r['Start_Timestamp']),int(r['End_Timestamp'])
ks=sorted((int(x['Start_Timestamp']),int(x['End_Timestamp'])) for x in csv.DictReader(open(d+'/run_kernel_trace.csv')))
inr=[k for k in ks if k[0]>=s and k[0]<=e]
print(d, 'region', (e-s)/1e3, 'head', (inr[0][0]-s)/1e3, 'tail', (e-inr[-1][1])/1e3, 'span', (inr[-1][1]-inr[0][0])/1e3, 'n', len(inr))

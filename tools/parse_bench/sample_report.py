"""Aggregate parse_bench -DH2J_SAMPLE addresses by source line and by function (innermost
inlined frame), via addr2line.  usage: sample_report.py BINARY SAMPLES [top]"""
import collections
import subprocess
import sys

binary, samples = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
addrs = [l.strip() for l in open(samples) if l.strip()]
count = collections.Counter(addrs)
uniq = list(count)
base = 0
for l in open('/proc/self/maps'):
    pass
out = subprocess.run(['addr2line', '-f', '-i', '-C', '-e', binary] + ['0x' + a for a in uniq],
                     capture_output=True, text=True).stdout.splitlines()
# addr2line -i prints several (func, line) pairs per address; re-run per address is slow, so use
# --addresses to delimit
out = subprocess.run(['addr2line', '-a', '-f', '-i', '-C', '-e', binary] + ['0x' + a for a in uniq],
                     capture_output=True, text=True).stdout.splitlines()
frames = {}
cur = None
i = 0
while i < len(out):
    if out[i].startswith('0x'):
        cur = out[i][2:].lstrip('0') or '0'
        frames[cur] = []
        i += 1
        continue
    frames[cur].append((out[i], out[i + 1].split(' (')[0]))
    i += 2
by_line = collections.Counter()
by_func = collections.Counter()
by_outer = collections.Counter()
n = len(addrs)
for a, c in count.items():
    fr = frames.get(a.lstrip('0') or '0') or [('?', '?')]
    func, line = fr[0]
    by_line[line.split('/')[-1] + '  ' + func[:50]] += c
    by_func[func[:90]] += c
    by_outer[fr[-1][0][:90]] += c
print('samples', n)
for title, ctr in (('innermost function', by_func), ('outermost function', by_outer), ('line', by_line)):
    print('--', title)
    for k, c in ctr.most_common(top):
        print('%6.2f%%  %s' % (100.0 * c / n, k))

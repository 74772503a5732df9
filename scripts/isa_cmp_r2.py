import sys
sys.path.insert(0,'/root/repo/scripts')
from isa_diff import kernels
for tu in ['capi','park']:
    a=kernels(f'/tmp/isa_r2/{tu}.s'); b=kernels(f'/tmp/isa_new/{tu}.s')
    bn={}
    for k,v in b.items():
        if 'k_persistent' in k:
            if k.endswith('ELb0EEEvNS_10RenderArgsEPy'): bn[k[:-len('ELb0EEEvNS_10RenderArgsEPy')]+'EEEvNS_10RenderArgsEPy']=v
        else: bn[k]=v
    same=diff=0
    for k in a:
        if k not in bn: print('missing',k); continue
        if a[k]==bn[k]: same+=1
        else: diff+=1; print('DIFF', len(a[k]), len(bn[k]), k[:90])
    print(tu, 'same',same,'diff',diff)

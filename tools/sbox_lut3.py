#!/usr/bin/env python3
# Generator (design tool, not run by tests): greedy packing of the Boyar-Peralta
# S-box circuit (tools/sbox_circuit.py) into 3-input LUTs = gfx950 v_bitop3_b32;
# prints the C body pasted into f-stack_amd/csrc/aes_bs.h sbox().
# Greedy LUT3 packing of the Boyar-Peralta S-box (from t2 on; y*, X7 are inputs)
import re
import os
src=open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'sbox_circuit.py')).read()
circ=src.split('CIRCUIT = """')[1].split('"""')[0].strip().splitlines()
gates=[]
for l in circ:
    lhs,rhs=[s.strip() for s in l.split('=')]
    rhs=rhs.replace('~','')          # NOT-free S-box (affine constant folded into keys)
    op='&' if '&' in rhs else '^'
    ins=[s.strip() for s in rhs.split(op)]
    gates.append((lhs,op,ins))
# linear layer handled by hand: everything named y* and t0,t1 is an input; x7 -> X7
lin={g for g,_,_ in gates if g.startswith('y') or g in ('t0','t1')}
body=[(g,op,[('X7' if i=='x7' else i) for i in ins]) for g,op,ins in gates if g not in lin]
outs={'s%d'%i for i in range(8)}
fan={}
for g,op,ins in body:
    for i in ins: fan[i]=fan.get(i,0)+1
# expression of each node as python lambda over its leaf inputs
expr={}   # node -> (leaves tuple, function)
def leafexpr(n): return ((n,), lambda env: env[n])
for g,op,ins in body:
    cands=[]
    for i in ins:
        if i in expr and fan.get(i,0)==1 and i not in outs:
            cands.append(i)
    # try to absorb as many single-fanout children as possible keeping <=3 leaves
    best=None
    import itertools
    for r in range(len(cands),-1,-1):
        for sub in itertools.combinations(cands,r):
            leaves=[]
            for i in ins:
                ls=expr[i][0] if i in sub else (i,)
                for x in ls:
                    if x not in leaves: leaves.append(x)
            if len(leaves)<=3:
                best=(sub,leaves);break
        if best: break
    sub,leaves=best
    fs=[(expr[i][1] if i in sub else (lambda env,i=i: env[i])) for i in ins]
    if op=='&': f=lambda env,fs=fs: fs[0](env)&fs[1](env)
    else: f=lambda env,fs=fs: fs[0](env)^fs[1](env)
    expr[g]=(tuple(leaves),f,sub)
absorbed=set()
for g,(l,f,sub) in expr.items(): absorbed|=set(sub)
emit=[g for g,_,_ in body if g not in absorbed]
pats=[0xf0,0xcc,0xaa]
lines=[]
for g in emit:
    leaves,f,sub=expr[g]
    env={x:pats[k] for k,x in enumerate(leaves)}
    tt=f(env)&0xff
    L=list(leaves)
    if len(L)==2:
        a,b=L
        # plain 2-input op when possible
        if tt==(0xf0^0xcc): lines.append('const uint32_t %s = %s ^ %s;'%(g,a,b)); continue
        if tt==(0xf0&0xcc): lines.append('const uint32_t %s = %s & %s;'%(g,a,b)); continue
        L.append(L[0]); env={x:pats[k] for k,x in enumerate(leaves)}
    lines.append('const uint32_t %s = __builtin_amdgcn_bitop3_b32(%s, %s, %s, 0x%02x);'%(g,L[0],L[1],L[2],tt))
print('// %d ops (%d gates, %d absorbed)'%(len(emit),len(body),len(absorbed)))
print('\n'.join(lines))

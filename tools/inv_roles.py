"""Per-role gemmx rates of one batched inverse from a tools/inv_trace.sh kernel trace (replays
chol.hip's panel / sub-panel loop):  python tools/inv_roles.py TRACE.csv.gz M BATCH"""
import csv,gzip,collections,sys
path,m,batch=sys.argv[1],int(sys.argv[2]),int(sys.argv[3])
rows=list(csv.DictReader(gzip.open(path,'rt')))
starts=[i for i,r in enumerate(rows) if 'hess_fill4' in r['Kernel_Name']]
seq=rows[starts[-1]:]
CP=1024 if m>6144 else 512;SP=256
calls=[]
def big(kind,M,N,K,upper):
    tiles=-(-M//128)*-(-N//128)//(2 if upper else 1)*batch
    if tiles>=64 and K>=128: calls.append((kind,M,N,K,upper))
P0=0
while P0<m:
    Pend=min(m,P0+CP); Q0=P0
    while Q0<Pend:
        Qend=min(Pend,Q0+SP)
        if Qend>=Pend: break
        K=Qend-Q0
        big('sub_trail',Pend-Qend,m-Qend,K,False); big('sub_trtri',Pend-Qend,Qend,K,False)
        Q0+=SP
    if Pend>=m: break
    K=Pend-P0; rest=m-Pend
    big('pan_trail',rest,rest,K,True); big('pan_trtri',rest,Pend,K,False)
    P0+=CP
calls.append(('lauum',m,m,m,True))
gx=[r for r in seq if 'gemmx' in r['Kernel_Name']]
print('gemmx launches',len(gx),'replayed',len(calls))
agg=collections.defaultdict(lambda:[0,0.0,0.0]); tot=0
for (kind,M,N,K,up),r in zip(calls,gx):
    d=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3
    fl=2.0*M*N*K*batch*(0.5 if up else 1)
    if kind=='lauum': fl=batch*m**3/3.0
    a=agg[kind]; a[0]+=1;a[1]+=d;a[2]+=fl; tot+=d
for k,(n,d,fl) in agg.items(): print(f'{k:10s} n={n:3d} {d/1e3:8.2f} ms {fl/d/1e6:7.1f} TF')
allk=sum((int(r['End_Timestamp'])-int(r['Start_Timestamp'])) for r in seq)/1e6
span=(int(seq[-1]['End_Timestamp'])-int(seq[0]['Start_Timestamp']))/1e6
print(f'gemmx {tot/1e3:.2f} ms, all kernels {allk:.2f} ms, span {span:.2f} ms, m^3 TF on span {batch*m**3/span/1e9:.1f}')
oth=collections.defaultdict(float)
for r in seq:
    if 'gemmx' not in r['Kernel_Name']: oth[r['Kernel_Name'][:70]]+=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6
for k,v in sorted(oth.items(),key=lambda x:-x[1]): print(f'{v:8.2f} {k}')

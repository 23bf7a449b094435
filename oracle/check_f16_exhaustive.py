import ctypes, numpy as np, time
R=ctypes.CDLL("oracle/_ref/libbpsr_ref.so"); P=ctypes.CDLL("oracle/liboracle.so")
R.bpsr_ref_create.restype=ctypes.c_void_p
R.bpsr_ref_sum.argtypes=[ctypes.c_void_p,ctypes.c_void_p,ctypes.c_void_p,ctypes.c_size_t,ctypes.c_int]
P.bpsr_oracle_sum.argtypes=[ctypes.c_void_p,ctypes.c_void_p,ctypes.c_size_t,ctypes.c_int,ctypes.c_int]
r=R.bpsr_ref_create()
src=np.arange(65536,dtype=np.uint16)
# extend with 7 tail elements: tail gets src values too
t=time.time(); bad=0
for d in range(0,65536):
    a=np.full(65536+7,d,dtype=np.uint16); b=np.concatenate([src,src[d*7%65536:(d*7%65536)+7] if d*7%65536+7<=65536 else src[:7]])
    a2=a.copy()
    R.bpsr_ref_sum(r,a.ctypes.data,b.ctypes.data,2*len(a),2)
    P.bpsr_oracle_sum(a2.ctypes.data,b.ctypes.data,2*len(a),2,1)
    if not np.array_equal(a,a2):
        idx=np.nonzero(a!=a2)[0]; bad+=len(idx)
        if bad<20: print(hex(d),[ (hex(b[i]),hex(a[i]),hex(a2[i])) for i in idx[:5]])
print("mismatch",bad,"time",time.time()-t)

import sys, numpy as np
sys.path.insert(0,'tests'); sys.path.insert(0,'image-webp_amd')
import oracle_lib as O, zwebp
ctx=zwebp.Context(0)
for (w,h,bpp,up) in [(17,9,4,0),(17,9,3,0),(33,31,4,0),(1920,1080,4,0),(17,9,4,1)]:
    mbw,mbh=(w+15)//16,(h+15)//16
    rng=np.random.default_rng(w*7919+h*31+bpp+5*up)
    y=rng.integers(0,256,mbw*16*mbh*16,dtype=np.uint8); u=rng.integers(0,256,mbw*8*mbh*8,dtype=np.uint8); v=rng.integers(0,256,mbw*8*mbh*8,dtype=np.uint8)
    got=zwebp.yuv_to_rgb(y,u,v,w,h,mbw*16,mbw*8,bpp,up,ctx=ctx).reshape(h,w,bpp)
    fn=O.yuv_to_rgb_fancy if up==0 else O.yuv_to_rgb_simple
    exp=fn(y,u,v,w,h,bpp).reshape(h,w,bpp)
    bad=np.argwhere((got!=exp).any(-1))
    print(w,h,bpp,up,"bad",len(bad), bad[:8].tolist(), [ (got[r,c].tolist(), exp[r,c].tolist()) for r,c in bad[:3]])

// Serial-chain probe of the boolean decoder: ns per decision for one stream
// and for two independent streams stepped in turn (instruction-level overlap).
// g++ -O3 -march=native tools/bool_chain_probe.cpp -o /tmp/probe && /tmp/probe
#include <cstdint>
#include <cstdio>
#include <chrono>
#include <vector>
#include <random>
struct BR {
    const uint8_t* d; size_t len, pos; uint64_t value; uint32_t range; int bits; bool eof;
    void init(const uint8_t* p, size_t n){d=p;len=n;pos=0;value=0;range=254;bits=-8;eof=false;load();}
    void load(){ size_t rem=len-pos; if(rem>=8){uint64_t v=0; for(int i=0;i<8;i++) v=(v<<8)|d[pos+i]; v>>=8; value=v|(value<<56); bits+=56; pos+=7;} else {value<<=8; bits+=8; eof=true;} }
    inline int bit(int prob){ if(bits<0) load(); uint32_t r=range; int p=bits; uint32_t split=(r*(uint32_t)prob)>>8; uint32_t v=(uint32_t)(value>>p); uint32_t b=v>split; uint32_t m=0u-b; uint32_t nr=((r-split)&m)|((split+1)&~m); value-=(uint64_t)((split+1)&m)<<p; int shift=7^(31^__builtin_clz(nr)); bits-=shift; range=(nr<<shift)-1; return (int)b; }
};
int main(){
    std::mt19937 g(1); std::vector<uint8_t> a(1<<22), b(1<<22), pr(4096);
    for(auto&x:a) x=g(); for(auto&x:b) x=g(); for(auto&x:pr) x=1+g()%254;
    const int N=3000000;
    for(int rep=0;rep<3;rep++){
    BR r1; r1.init(a.data(),a.size()); int acc=0;
    auto t0=std::chrono::steady_clock::now();
    for(int i=0;i<N;i++){ acc+=r1.bit(pr[(i+acc)&4095]); }
    double t1=std::chrono::duration<double,std::nano>(std::chrono::steady_clock::now()-t0).count()/N;
    BR s1,s2; s1.init(a.data(),a.size()); s2.init(b.data(),b.size()); int a1=0,a2=0;
    t0=std::chrono::steady_clock::now();
    for(int i=0;i<N/2;i++){ a1+=s1.bit(pr[(i+a1)&4095]); a2+=s2.bit(pr[(i+a2+7)&4095]); }
    double t2=std::chrono::duration<double,std::nano>(std::chrono::steady_clock::now()-t0).count()/N;
    printf("1 stream %.2f ns/bit, 2 interleaved %.2f ns/bit (%d %d %d)\n",t1,t2,acc,a1,a2);}
}

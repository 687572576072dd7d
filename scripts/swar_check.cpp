// Host check of the tile kernel's four-bytes-a-step image-reference scan (kernels.hip parse_image,
// KW_SWAR_PARSE) against the byte loop it replaces, on 2M random strings over the delimiter alphabet.
// g++ -O2 -o /tmp/swar_check scripts/swar_check.cpp && /tmp/swar_check
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <algorithm>
const uint32_t NONE=0xffffffffu;
struct R{uint32_t at,s0,s1,lc;bool dc;};
R ref(const uint8_t* bytes,uint32_t b,uint32_t e){R r{NONE,NONE,NONE,NONE,false};
 for(uint32_t q=b;q<e;++q){uint8_t c=bytes[q]; if(c=='@'){r.at=q;break;}
  if(c=='/'){if(r.s0==NONE)r.s0=q;else if(r.s1==NONE)r.s1=q;} else if(c==':'){r.lc=q;if(r.s0==NONE)r.dc=true;} else if(c=='.'){if(r.s0==NONE)r.dc=true;}}
 return r;}
R swar(const uint8_t* bytes,uint32_t b,uint32_t e){R r{NONE,NONE,NONE,NONE,false};
 auto eqb=[](uint32_t x,uint32_t c4)->uint32_t{uint32_t y=x^c4;return ~(((y&0x7F7F7F7Fu)+0x7F7F7F7Fu)|y|0x7F7F7F7Fu);};
 for(uint32_t p0=b&~3u;p0<e;p0+=4u){uint32_t w;memcpy(&w,bytes+p0,4);
  uint32_t lo=p0<b?b-p0:0u, hi=std::min(4u,e-p0);
  uint32_t vm=(0x80808080u<<(8u*lo))&(hi>=4u?0xffffffffu:((1u<<(8u*hi))-1u));
  uint32_t m_at=eqb(w,0x40404040u)&vm,m_sl=eqb(w,0x2f2f2f2fu)&vm,m_co=eqb(w,0x3a3a3a3au)&vm,m_dt=eqb(w,0x2e2e2e2eu)&vm;
  if(m_at){uint32_t keep=(1u<<__builtin_ctz(m_at))-1u; r.at=p0+__builtin_ctz(m_at)/8u; m_sl&=keep;m_co&=keep;m_dt&=keep;}
  if(m_co) r.lc=p0+(31u-__builtin_clz(m_co))/8u;
  if(r.s0==NONE){uint32_t before=m_sl?(1u<<__builtin_ctz(m_sl))-1u:0xffffffffu; if((m_co|m_dt)&before) r.dc=true; if(m_sl){r.s0=p0+__builtin_ctz(m_sl)/8u; m_sl&=m_sl-1u;}}
  if(r.s1==NONE&&m_sl) r.s1=p0+__builtin_ctz(m_sl)/8u;
  if(m_at)break;}
 return r;}
int main(){std::mt19937 g(1);const char al[]="@/:.ab\x00\x01\x7f\x80\xff";uint8_t buf[128];long bad=0;
 for(int it=0;it<2000000;++it){for(auto&c:buf)c=al[g()%11]; uint32_t b=g()%40,e=b+g()%60; R x=ref(buf,b,e),y=swar(buf,b,e);
  if(x.at!=y.at||x.s0!=y.s0||x.s1!=y.s1||x.lc!=y.lc||x.dc!=y.dc){if(bad<5)printf("mismatch b=%u e=%u\n",b,e);++bad;}}
 printf("mismatches %ld\n",bad);}

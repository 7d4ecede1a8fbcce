/* Check for k_orb's sincosf_glibc_lanes: glibc 2.35's sinf/cosf small-argument branch (y < 0.75: the
   polynomials on y unreduced, (y, 1) below top 0x397) and its reduced branch (n = round(y 2/pi) = 0 there)
   return the same floats for every float y in [0, 0.75).  Same double FMA expressions as the kernel.
   build: gcc -O2 -ffp-contract=off -o /tmp/sincos_paths tools/dbg/sincos_paths.c -lm  (prints "bad 0") */
#include <stdio.h>
#include <math.h>
#include <string.h>
#include <stdint.h>
static const double hpi_inv = 0x1.45f306dc9c883p+23, hpi = 0x1.921fb54442d18p+0;
static const double c0 = 0x1p+0, c1 = -0x1.ffffffd0c621cp-2, c2 = 0x1.55553e1068f19p-5, c3 = -0x1.6c087e89a359dp-10, c4 = 0x1.99343027bf8c3p-16;
static const double s1 = -0x1.555545995a603p-3, s2 = 0x1.1107605230bc4p-7, s3 = -0x1.994eb3774cf24p-13;
static float sinp(double x, double x2){ double x3=x*x2, a=fma(x2,s3,s2), x5=x2*x3, s=fma(x3,s1,x); return (float)fma(x5,a,s);}
static float cosp(double x2){ double x4=x2*x2, a=fma(x2,c1,c0), b=fma(x2,c4,c3), x6=x2*x4; double c=fma(x4,c2,a); return (float)fma(x6,b,c);}
static void small(float y, float*sn, float*cs){ unsigned u; memcpy(&u,&y,4); unsigned top=(u>>20)&0x7ff; double x=y, x2=x*x;
  *sn = top<=0x397 ? y : sinp(x,x2); *cs = top<=0x397 ? 1.0f : cosp(x2);}
static void red(float y, float*sn, float*cs){ double x=y; double r=x*hpi_inv; int n=(((int)r)+0x800000)>>24; x=fma(-(double)n,hpi,x);
  double x2=x*x; double xs=((n^(n>>1))&1)?-x:x; float cp=((n>>1)&1)?-cosp(x2):cosp(x2); float sp=sinp(xs,x2); *sn=(n&1)?cp:sp; *cs=(n&1)?sp:cp;}
int main(){ long bad=0; for(uint32_t u=0; u<=0x3F3FFFFFu; ++u){ float y; memcpy(&y,&u,4); float a,b,c,d; small(y,&a,&b); red(y,&c,&d);
  if(memcmp(&a,&c,4)||memcmp(&b,&d,4)){ if(bad<5) printf("diff %08x %a %a | %a %a\n",u,a,b,c,d); ++bad;} }
  printf("bad %ld\n",bad); return 0;}

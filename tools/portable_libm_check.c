/* Accuracy of csrc/rt/portable_libm.h against glibc (the diagnostic libm of tests/test_gpu_libm_isolation.py):
 * max abs error of sin on [-200, 200], rel error of log on (0, 1], abs error of atan2 / acos on [-1, 1].
 * usage: portable_libm_check  (prints one line; tests/test_divisions.py bounds it) */
#include "portable_libm.h"
#include <stdio.h>
#include <stdlib.h>
int main(){ double ms=0,ml=0,ma=0,mc=0; srand(1);
 for(int i=0;i<2000000;i++){ double x=((double)rand()/RAND_MAX-0.5)*400; double u=(double)rand()/RAND_MAX;
  double y=((double)rand()/RAND_MAX-0.5)*2, z=((double)rand()/RAND_MAX-0.5)*2;
  double e=fabs(pl_sin(x)-sin(x)); if(e>ms)ms=e;
  if(u>0){e=fabs(pl_log(u)-log(u))/fabs(log(u)); if(e>ml)ml=e;}
  e=fabs(pl_atan2(y,z)-atan2(y,z)); if(e>ma)ma=e;
  e=fabs(pl_acos(y)-acos(y)); if(e>mc)mc=e; }
 printf("max abs err sin %.3g  rel log %.3g  atan2 %.3g  acos %.3g  log(0)=%g pow5(0.5)=%.17g\n",ms,ml,ma,mc,pl_log(0.0),pl_pow5(0.5)); }

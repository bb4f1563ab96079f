// tools/walk_windows_sim.c — host simulation of the LP walk's 32-byte windows (4 slots, never crossing a
// 128-byte line) on a load-1/4 table of the reference hash: windows per probe row walking every run
// to its end vs ending a row at its match (distinct keys).  gcc -O2 -o /tmp/wsim tools/walk_windows_sim.c && /tmp/wsim 24
// windows per probe row for the walk: runs from home to first empty, 4-slot windows not crossing
// 16-slot lines (s = min(cur, line_end-4)); with / without early exit on match (distinct keys)
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
static uint64_t mh(uint64_t x){x^=x>>32;x*=0xd6e8feb86659fd93ULL;x^=x>>32;x*=0xd6e8feb86659fd93ULL;x^=x>>32;return x;}
static uint64_t sm(uint64_t *s){uint64_t z=(*s+=0x9e3779b97f4a7c15ULL);z=(z^(z>>30))*0xbf58476d1ce4e5b9ULL;z=(z^(z>>27))*0x94d049bb133111ebULL;return z^(z>>31);}
int main(int argc,char**argv){
  int kb=atoi(argv[1]); uint64_t nk=1ull<<kb, size=nk*4, mask=size-1;
  int64_t *t=malloc(size*8); for(uint64_t i=0;i<size;i++)t[i]=-1;
  for(uint64_t k=0;k<nk;k++){uint64_t h=mh(k)&mask; while(t[h]!=-1)h=(h+1)&mask; t[h]=k;}
  uint64_t seed=42; double w_full=0,w_early=0,slots=0; uint64_t n=1<<24;
  for(uint64_t i=0;i<n;i++){uint64_t key=sm(&seed)%nk; uint64_t cur=mh(key)&mask; int wf=0,we=0,found=0; uint64_t exam=0;
    for(;;){uint64_t s=cur; if(s>size-4)s=size-4; uint64_t lim=(s&~15ull)+12; if(s>lim)s=lim;
      wf++; if(!found)we++;
      int end=0; for(uint64_t j=cur;j<s+4;j++){exam++; if(t[j]==-1){end=1;break;} if(t[j]==(int64_t)key)found=1;}
      if(end)break; cur=(s+4)&mask;}
    w_full+=wf; w_early+=we; slots+=exam;}
  printf("kb %d: windows/row full %.4f early-exit %.4f, slots examined %.4f\n",kb,w_full/n,w_early/n,slots/n);
}

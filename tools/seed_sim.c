// Seeded-chunk simulation (np_sampler.hip "Seeded chunks"): K evenly spread entry
// states parsed through random 32-bit words with numpy's random_interval rule; reports the
// trajectory-draws of a chunk, the trajectories left after 2^12..2^19 draws, and how many
// draws a random true entry (or the worst of four) needs to meet a seed trajectory at
// checkpoints CK draws apart.  gcc -O2 -o /tmp/seed_sim tools/seed_sim.c
//   /tmp/seed_sim <n1> <K> <trials> <chunk draws> <CK> <seed>
// K seeds: trajectory-draw cost and extension (true-entry merge) time at checkpoint granularity CK
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
static uint64_t rs;
static inline uint32_t nxt(void){ rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return (uint32_t)(rs >> 11); }
static inline uint32_t msk(uint32_t i){ return 0xffffffffu >> __builtin_clz(i); }
static inline uint32_t step(uint32_t s, uint32_t w, uint32_t n1){ if((w & msk(s)) <= s){ s--; if(!s) s=n1; } return s; }
static int cmpi(const void*a,const void*b){return *(int*)a-*(int*)b;}
int main(int argc,char**argv){
  int n1=atoi(argv[1]),K=atoi(argv[2]),trials=atoi(argv[3]),L=atoi(argv[4]),CK=atoi(argv[5]);
  rs = 0x9e3779b97f4a7c15ull ^ ((uint64_t)K<<20) ^ (uint64_t)atoi(argv[6]);
  uint32_t *w=malloc(4*(size_t)L), st[4096]; int *ee=malloc(4*trials), *e4=malloc(4*trials);
  double tdraws=0; double mAt[8]={0}; int at[8]={4096,16384,65536,131072,262144,524288,0,0};
  for(int t=0;t<trials;t++){
    for(int k=0;k<L;k++) w[k]=nxt();
    int m=K; for(int k=0;k<m;k++) st[k]=n1-(uint32_t)((long long)k*n1/m);
    uint32_t xs[4]; for(int g=0;g<4;g++){ uint32_t x=1+nxt()%n1; for(int k=0;k<50000;k++) x=step(x,nxt(),n1); xs[g]=x; }
    int text[4]={-1,-1,-1,-1};
    for(int d=0;d<L;d++){
      uint32_t wd=w[d];
      for(int k=0;k<m;k++) st[k]=step(st[k],wd,n1);
      for(int g=0;g<4;g++) if(text[g]<0) xs[g]=step(xs[g],wd,n1);
      tdraws+=m;
      if(((d+1)%CK)==0){
        int mm=0; for(int k=0;k<m;k++){ uint32_t p=st[(k+m-1)%m]; if(m>1 && st[k]==p) continue; st[mm++]=st[k]; }
        if(mm==0) mm=1; m=mm;
        for(int g=0;g<4;g++) if(text[g]<0) for(int k=0;k<m;k++) if(st[k]==xs[g]){text[g]=d+1;break;}
      }
      for(int a=0;a<6;a++) if(d+1==at[a]) mAt[a]+=m;
    }
    for(int g=0;g<4;g++) if(text[g]<0) text[g]=L;
    ee[t]=text[0]; int mx=0; for(int g=0;g<4;g++) if(text[g]>mx) mx=text[g]; e4[t]=mx;
  }
  qsort(ee,trials,4,cmpi); qsort(e4,trials,4,cmpi);
  printf("K=%d CK=%d: traj-draws/chunk %.3g  m@4k,16k,64k,128k,256k,512k:",K,CK,tdraws/trials);
  for(int a=0;a<6;a++) printf(" %.1f",mAt[a]/trials);
  printf("\n  ext1 p50 %d p90 %d p99 %d p99.5 %d max %d | max-of-4 p50 %d p90 %d p99 %d max %d\n",
    ee[trials/2],ee[trials*9/10],ee[trials*99/100],ee[trials*995/1000],ee[trials-1],e4[trials/2],e4[trials*9/10],e4[trials*99/100],e4[trials-1]);
}

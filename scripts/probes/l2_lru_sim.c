// LRU model of the SpMM gather stream per XCD (4 MiB, 16-way, 128-B lines):
// rows of each XCD range processed `conc` at a time, edge by edge round
// robin (the concurrency of the resident waves); rows optionally sorted by
// (window, -length).  Input: /tmp/sim/rp.bin (int64 rowptr), /tmp/sim/col.bin
// (int32 col) written by scripts/l2_sim.py.
// Usage: l2_lru_sim n nnz B window conc
// LRU L2 sim: per XCD, rows (not chunks) of the XCD's contiguous ranges,
// processed in order of (window, -len); 2 rows interleaved edge by edge (pairs).
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
typedef struct { int64_t *tag; int64_t *age; int sets, ways; int64_t clk; } Cache;
static void cinit(Cache*c,int64_t bytes,int line,int ways){c->ways=ways;c->sets=bytes/line/ways;c->tag=malloc(8L*c->sets*ways);c->age=calloc((size_t)c->sets*ways,8);for(int64_t i=0;i<(int64_t)c->sets*ways;i++)c->tag[i]=-1;c->clk=0;}
static int acc(Cache*c,int64_t line){int64_t s=line% c->sets;int64_t*t=c->tag+s*c->ways,*a=c->age+s*c->ways;c->clk++;int lru=0;for(int w=0;w<c->ways;w++){if(t[w]==line){a[w]=c->clk;return 1;}if(a[w]<a[lru])lru=w;}t[lru]=line;a[lru]=c->clk;return 0;}
static int64_t *RP; static int WIN;
static int cmp(const void*x,const void*y){int a=*(int*)x,b=*(int*)y;int wa=a/WIN,wb=b/WIN;if(wa!=wb)return wa-wb;int la=RP[a+1]-RP[a],lb=RP[b+1]-RP[b];if(la!=lb)return lb-la;return a-b;}
int main(int argc,char**argv){
  int64_t n=atoll(argv[1]),nnz=atoll(argv[2]);int B=atoi(argv[3]);WIN=atoi(argv[4]);int conc=atoi(argv[5]);
  int64_t*rp=malloc(8*(n+1));int32_t*col=malloc(4*nnz);RP=rp;
  FILE*f=fopen("/tmp/sim/rp.bin","rb");if(fread(rp,8,n+1,f)){};fclose(f);f=fopen("/tmp/sim/col.bin","rb");if(fread(col,4,nnz,f)){};fclose(f);
  int64_t hits=0,miss=0;
  int *rows=malloc(4*n);
  for(int x=0;x<8;x++){
    Cache c; cinit(&c,4L<<20,128,16);
    int m=0;
    for(int r=x*B/8;r<(x+1)*B/8;r++)rows[m++]=r;
    int64_t nb=n-B; for(int64_t r=B+x*nb/8;r<B+(x+1)*nb/8;r++)rows[m++]=r;
    if(WIN>0) qsort(rows,m,4,cmp);
    // conc rows in flight, round-robin one edge each (approximates concurrency)
    int *cur=malloc(4*conc),*cr=malloc(4*conc); int next=0,active=0;
    for(int i=0;i<conc&&next<m;i++){cr[i]=rows[next++];cur[i]=rp[cr[i]];active++;}
    for(int i=conc>m?m:conc;i<conc;i++)cr[i]=-1;
    while(active>0){
      for(int i=0;i<conc;i++){ if(cr[i]<0)continue;
        if(cur[i]>=rp[cr[i]+1]){ if(next<m){cr[i]=rows[next++];cur[i]=rp[cr[i]];} else {cr[i]=-1;active--;continue;} if(cur[i]>=rp[cr[i]+1]) continue; }
        int64_t base=(int64_t)col[cur[i]]*4; for(int l=0;l<4;l++){if(acc(&c,base+l))hits++;else miss++;}
        cur[i]++;
      }
    }
    free(c.tag);free(c.age);free(cur);free(cr);
  }
  printf("win=%d conc=%d hit=%.3f missMB=%.1f\n",WIN,conc,(double)hits/(hits+miss),miss*128/1e6);
}

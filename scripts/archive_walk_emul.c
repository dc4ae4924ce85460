// CPU emulation of the archive decoder's boundary discovery (nxg_archive.hip: spec walks, chain,
// repair walkers, stitch) on an archive batch file, checked against a sequential walk. Used to
// validate the algorithm before the GPU version; usage: archive_walk_emul <batch.bin> <chunk>.
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
static const uint8_t* B; static uint64_t W;
static int var(uint64_t* p, uint64_t* v){uint64_t x=0;for(int i=0;i<10;i++){if(*p>=W)return 1;uint8_t b=B[(*p)++];x|=(uint64_t)(b&0x7f)<<(7*i);if(b<0x80){*v=x;return 0;}}return 1;}
static int fixsz(int t){switch(t){case 0:case 2:case 8:return 4;case 4:case 6:case 9:return 8;case 10:case 11:return 12;case 14:case 15:case 16:case 17:return 0;case 20:return 16;case 23:case 24:return 1;case 25:case 26:return 2;default:return -1;}}
static int val(uint64_t* p,int d){ if(d>32)return 1; if(*p>=W)return 1; int t=B[(*p)++]; uint64_t v;
 int f=fixsz(t); if(f>=0){ if(W-*p<(uint64_t)f)return 1; *p+=f; return 0;}
 switch(t){case 1:case 3:case 5:case 7: return var(p,&v);
 case 12: case 13: case 18: if(var(p,&v))return 1; if(v>W-*p)return 1; *p+=v; return 0;
 case 19: case 21: { if(var(p,&v))return 1; uint64_t u=t==19?16:32; if(v>(1ull<<31)/u || v*u>((W-*p)<<8)) return 1; uint64_t k=t==19?v:2*v; for(uint64_t i=0;i<k;i++) if(val(p,d+1))return 1; return 0;}
 case 22: return val(p,d+1);
 case 27: { if(var(p,&v))return 1; if(v<1)return 1; *p+=v-1; if(*p>W) return 1; return 0;}
 default: return 1;}}
static int item(uint64_t* p){uint64_t id; if(var(p,&id))return 1; if(*p>=W)return 1; if(B[*p]==0x40){(*p)++;return 0;} return val(p,0);}
#define ERR (~0ull)
static uint64_t p0, CH, nch;
static uint64_t chain(uint64_t k, uint64_t e){ if(e==ERR) return ERR; uint64_t s=p0+k*CH, lim=s+CH<W?s+CH:W, q=e; while(q<lim){uint64_t r=q; if(item(&r)) return ERR; q=r;} return q; }
typedef struct { uint64_t exit; uint32_t from,count; } Rec;
int main(int argc,char**argv){ FILE*f=fopen(argv[1],"rb"); fseek(f,0,2); W=ftell(f); fseek(f,0,0); uint8_t*b=malloc(W); if(fread(b,1,W,f)!=W) return 2; B=b; CH=atoll(argv[2]);
 uint64_t cnt; p0=0; var(&p0,&cnt); nch=W/CH+2;
 uint64_t *xg=malloc(nch*8),*y=malloc(nch*8),*tx=malloc(nch*8);
 { uint64_t e=p0; for(uint64_t k=0;k<nch;k++){ e=chain(k,e); tx[k]=e; } }
 for(uint64_t k=0;k<nch;k++){ uint64_t s=p0+k*CH; if(s>=W){xg[k]=W;continue;} uint64_t lim=s+CH<W?s+CH:W; uint64_t q=s; while(q<lim){ uint64_t r=q; if(item(&r)) q++; else q=r; } xg[k]=q; }
 for(uint64_t k=0;k<nch;k++) y[k]=chain(k, k?xg[k-1]:p0);
 uint64_t nw=0; uint32_t* st=malloc(nch*4); for(uint64_t k=0;k+1<nch;k++) if(y[k]!=xg[k] && y[k]!=ERR) st[nw++]=k+1;
 Rec* rec=malloc(nw*16*sizeof(Rec)); uint32_t *nrec=calloc(nw,4),*last=calloc(nw,4),*state=calloc(nw,4); uint64_t maxwalk=0;
 for(uint64_t i=0;i<nw;i++){ uint64_t j=st[i], e=y[j-1]; uint32_t nr=0,walks=0,s2=1; Rec* r=rec+i*16;
   while(nr<16 && walks<8){ uint64_t s=p0+j*CH, lim=s+CH<W?s+CH:W;
     if(e>=lim && j+1<nch){ uint64_t home=(e-p0)/CH; if(home>nch-1) home=nch-1; r[nr++]=(Rec){e,(uint32_t)j,(uint32_t)(home-j)}; j=home; if(e==xg[j-1]){s2=0;break;} continue; }
     uint64_t x=chain(j,e); walks++; r[nr++]=(Rec){x,(uint32_t)j,1}; if(x==ERR){s2=2;break;} if(j+1>=nch || x==xg[j]){s2=0;break;} e=x; j++; }
   nrec[i]=nr; last[i]=r[nr-1].from+r[nr-1].count-1; state[i]=s2; if(walks>maxwalk)maxwalk=walks; }
 int64_t lst=-2; uint64_t resume=nch, real=0;
 for(uint64_t i=0;i<nw;i++){ if((int64_t)st[i]<=lst+1) continue; real++; Rec* r=rec+i*16; for(uint32_t q=0;q<nrec[i];q++) for(uint32_t j=r[q].from;j<r[q].from+r[q].count;j++) y[j]=r[q].exit;
   if(state[i]==1){ resume=last[i]+1; break;} if(state[i]==2) break; lst=last[i]; }
 if(resume<nch){ uint64_t e=y[resume-1]; for(uint64_t k=resume;k<nch;k++){ e=chain(k,e); y[k]=e; } }
 uint64_t bad=0; for(uint64_t k=0;k<nch;k++) if(y[k]!=tx[k]) bad++;
 printf("CH=%lu nch=%lu walkers=%lu real=%lu maxwalk=%lu resume=%lu mismatched=%lu\n",CH,nch,nw,real,maxwalk,resume,bad); return 0;}

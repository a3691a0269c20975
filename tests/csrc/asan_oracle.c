/* The oracle (test infrastructure) under ASan/UBSan: every ec_encode_data kernel
 * family (AVX2, AVX-512, GFNI) against ec_encode_data_base on random shapes and
 * ragged lengths, 1-3 threads, and the encodeData flow in every family and local
 * mode (tests/test_sanitize.py). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
void orc_gen_cauchy1_matrix(uint8_t*,int,int);
void orc_init_tables_kind(int,int,int,const uint8_t*,uint8_t*);
void orc_encode_data_kind(int,int,int,int,const uint8_t*,uint8_t**,uint8_t**);
void orc_encode_data_base(int,int,int,const uint8_t*,uint8_t**,uint8_t**);
void orc_init_tables(int,int,const uint8_t*,uint8_t*);
void orc_encode_data_mt_kind(int,int,int,int,const uint8_t*,uint8_t**,uint8_t**,int);
void* orc_codec_new(char,int,int,int,int,int,int);
void orc_nc_encode_mt_kind(void*,uint8_t**,uint8_t**,int,int,int,int);
void orc_codec_free(void*);
int main(){
  srand(1);
  int lens[]={1,17,63,64,65,127,128,1000,4096,4097};
  for(int t=0;t<200;t++){
    int k=1+rand()%40, m=1+rand()%13, len=lens[rand()%10];
    uint8_t*a=malloc((k+m)*k); orc_gen_cauchy1_matrix(a,k+m,k);
    uint8_t*tb=malloc(32*k*m), *tb0=malloc(32*k*m);
    orc_init_tables(k,m,a+k*k,tb0);
    uint8_t*src[64],*d0[16],*d1[16];
    for(int j=0;j<k;j++){src[j]=malloc(len);for(int i=0;i<len;i++)src[j][i]=rand();}
    for(int j=0;j<m;j++){d0[j]=malloc(len);d1[j]=malloc(len);}
    orc_encode_data_base(len,k,m,tb0,src,d0);
    for(int kind=1;kind<=3;kind++){
      orc_init_tables_kind(kind,k,m,a+k*k,tb);
      orc_encode_data_mt_kind(kind,len,k,m,tb,src,d1,1+rand()%3);
      for(int j=0;j<m;j++) if(memcmp(d0[j],d1[j],len)){printf("MISMATCH kind %d k %d m %d len %d\n",kind,k,m,len);return 1;}
    }
    for(int j=0;j<k;j++)free(src[j]); for(int j=0;j<m;j++){free(d0[j]);free(d1[j]);}
    free(a);free(tb);free(tb0);
  }
  /* codec flow, every kind, literal and XOR */
  for(int kind=0;kind<=3;kind++) for(int lit=0;lit<2;lit++){
    int k=29,m=3,r=8,len=5000; void*c=orc_codec_new('C',k,m,r,len,1,0);
    uint8_t*d[29],*p[8]; for(int j=0;j<k;j++){d[j]=malloc(len);memset(d[j],j+1,len);} for(int j=0;j<m+4;j++)p[j]=malloc(len);
    orc_nc_encode_mt_kind(c,d,p,lit,3,len,kind);
    for(int j=0;j<k;j++)free(d[j]); for(int j=0;j<m+4;j++)free(p[j]); orc_codec_free(c);
  }
  printf("asan oracle ok\n"); return 0;
}

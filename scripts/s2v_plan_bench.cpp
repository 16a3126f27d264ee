// Round 6: CPU microbenchmark of one sent2vec minibatch plan (1M Zipf(1M) tokens): hash-map
// counting, std::sort vs the LSD radix sort of (key, count), the unigram run starts with and
// without the memoised pow(c, 0.75).  g++ -O2 -o /tmp/plan scripts/s2v_plan_bench.cpp && /tmp/plan
#include <cstdint>
#include <vector>
#include <algorithm>
#include <cmath>
#include <chrono>
#include <cstdio>
#include <random>
static inline uint64_t fmix64(uint64_t k){k^=k>>33;k*=0xff51afd7ed558ccdULL;k^=k>>33;k*=0xc4ceb9fe1a85ec53ULL;k^=k>>33;return k;}
struct FlatMap64 {
  std::vector<uint64_t> k; std::vector<int32_t> v; std::vector<uint32_t> st; uint32_t gen=1; uint64_t mask=0; size_t n=0;
  explicit FlatMap64(size_t cap=16){reset(cap);}
  void reset(size_t cap){size_t c=16;while(c<2*cap)c<<=1;k.assign(c,0);v.assign(c,0);st.assign(c,0);mask=c-1;n=0;gen=1;}
  void clear(){if(++gen==0){std::fill(st.begin(),st.end(),0u);gen=1;}n=0;}
  void grow(){std::vector<uint64_t> ok; std::vector<int32_t> ov; std::vector<uint32_t> os; ok.swap(k); ov.swap(v); os.swap(st); uint32_t og=gen; size_t c=(mask+1)*2; k.assign(c,0);v.assign(c,0);st.assign(c,0);mask=c-1;n=0;gen=1;
    for(size_t i=0;i<ok.size();i++) if(os[i]==og) at(ok[i])=ov[i];}
  int32_t &at(uint64_t key,bool*fresh=nullptr){ if(2*(n+1)>mask+1)grow(); uint64_t i=fmix64(key)&mask; while(st[i]==gen){ if(k[i]==key){if(fresh)*fresh=false;return v[i];} i=(i+1)&mask;} st[i]=gen;k[i]=key;v[i]=0;n++; if(fresh)*fresh=true; return v[i];}
};
void starts(const std::vector<std::pair<uint64_t,int32_t>>&vc,uint64_t T,std::vector<uint64_t>&st){
  const size_t V=vc.size(); double pw=0; for(auto&kc:vc) pw+=std::pow(kc.second,0.75); st.assign(V+1,T); st[0]=0; double d1=std::pow(vc[0].second,0.75)/pw;
  for(size_t i=0;i+1<V;i++){ const uint64_t lo=st[i]; auto pred=[&](uint64_t a){return (int64_t)a/(double)T>d1;}; uint64_t a=(uint64_t)std::max<double>((double)lo,std::floor(d1*(double)T)); if(a>T)a=T; while(a>lo&&pred(a-1))a--; while(a<T&&!pred(a))a++; if(a>=T)break; st[i+1]=a+1; d1+=std::pow(vc[i+1].second,0.75)/pw;}
}
struct FlatMapAoS {
  struct Slot { uint64_t k; int32_t v; uint32_t g; };
  std::vector<Slot> t; uint32_t gen=1; uint64_t mask=0; size_t n=0;
  explicit FlatMapAoS(size_t cap=16){reset(cap);}
  void reset(size_t cap){size_t c=16;while(c<2*cap)c<<=1;t.assign(c,Slot{0,0,0});mask=c-1;n=0;gen=1;}
  void clear(){if(++gen==0){for(auto&x:t)x.g=0;gen=1;}n=0;}
  void grow(){std::vector<Slot> o; o.swap(t); uint32_t og=gen; size_t c=(mask+1)*2; t.assign(c,Slot{0,0,0}); mask=c-1;n=0;gen=1; for(auto&x:o) if(x.g==og) at(x.k)=x.v;}
  int32_t &at(uint64_t key,bool*fresh=nullptr){ if(2*(n+1)>mask+1)grow(); uint64_t i=fmix64(key)&mask; while(t[i].g==gen){ if(t[i].k==key){if(fresh)*fresh=false;return t[i].v;} i=(i+1)&mask;} t[i].g=gen;t[i].k=key;t[i].v=0;n++; if(fresh)*fresh=true; return t[i].v;}
};
// LSD radix sort of (key, count) by key, 8-bit digits, skipping digits every key shares
void radix_sort(std::vector<std::pair<uint64_t,int32_t>>&a, std::vector<std::pair<uint64_t,int32_t>>&tmp){
  const size_t n=a.size(); tmp.resize(n);
  for(int sh=0;sh<64;sh+=8){ size_t h[256]={0}; for(auto&x:a) h[(x.first>>sh)&255]++;
    bool one=false; for(int b=0;b<256;b++) if(h[b]==n){one=true;break;} if(one) continue;
    size_t o=0; for(int b=0;b<256;b++){size_t c=h[b];h[b]=o;o+=c;}
    for(auto&x:a) tmp[h[(x.first>>sh)&255]++]=x; a.swap(tmp);}
}
static double pw75[4096];
void starts2(const std::vector<std::pair<uint64_t,int32_t>>&vc,uint64_t T,std::vector<uint64_t>&st){
  auto P=[](int32_t c){return (c>=0&&c<4096)?pw75[c]:std::pow(c,0.75);};
  const size_t V=vc.size(); double pw=0; for(auto&kc:vc) pw+=P(kc.second); st.assign(V+1,T); st[0]=0; double d1=P(vc[0].second)/pw;
  for(size_t i=0;i+1<V;i++){ const uint64_t lo=st[i]; auto pred=[&](uint64_t a){return (int64_t)a/(double)T>d1;}; uint64_t a=(uint64_t)std::max<double>((double)lo,std::floor(d1*(double)T)); if(a>T)a=T; while(a>lo&&pred(a-1))a--; while(a<T&&!pred(a))a++; if(a>=T)break; st[i+1]=a+1; d1+=P(vc[i+1].second)/pw;}
}
int main(){ for(int c=0;c<4096;c++) pw75[c]=std::pow(c,0.75);
  const int V=1000000; const size_t NT=1024000;
  std::vector<double> cdf(V); double s=0; for(int i=0;i<V;i++){s+=1.0/(i+1);cdf[i]=s;} for(auto&c:cdf)c/=s;
  std::mt19937_64 g(5); std::uniform_real_distribution<double> u(0,1);
  std::vector<uint64_t> tok(NT); for(auto&t:tok){ t=std::lower_bound(cdf.begin(),cdf.end(),u(g))-cdf.begin()+1; }
  FlatMap64 fq(1<<16); std::vector<uint64_t> first; std::vector<std::pair<uint64_t,int32_t>> vc; std::vector<uint64_t> st;
  for(int rep=0;rep<3;rep++){
  auto t0=std::chrono::steady_clock::now();
  fq.clear(); first.clear();
  for(size_t i=0;i<NT;i++){bool fr=false; fq.at(tok[i],&fr)++; if(fr) first.push_back(tok[i]);}
  auto t1=std::chrono::steady_clock::now();
  vc.clear(); for(auto k:first) vc.emplace_back(k,fq.at(k)); std::sort(vc.begin(),vc.end());
  auto t2=std::chrono::steady_clock::now();
  starts(vc,100000000ULL,st);
  auto t3=std::chrono::steady_clock::now();
  std::vector<std::pair<uint64_t,int32_t>> vc2, tmp; for(auto k:first) vc2.emplace_back(k,fq.at(k));
  auto t4=std::chrono::steady_clock::now(); radix_sort(vc2,tmp); auto t5=std::chrono::steady_clock::now();
  std::vector<uint64_t> st2; starts2(vc2,100000000ULL,st2); auto t6=std::chrono::steady_clock::now();
  FlatMapAoS fa(1<<16); fa.clear(); std::vector<uint64_t> f2; auto t7=std::chrono::steady_clock::now();
  for(size_t i=0;i<NT;i++){bool fr=false; fa.at(tok[i],&fr)++; if(fr) f2.push_back(tok[i]);}
  auto t8=std::chrono::steady_clock::now(); fa.clear(); f2.clear(); auto t9=std::chrono::steady_clock::now();
  for(size_t i=0;i<NT;i++){bool fr=false; fa.at(tok[i],&fr)++; if(fr) f2.push_back(tok[i]);}
  auto t10=std::chrono::steady_clock::now();
  printf("aos count %.2f (grown %.2f) ms equal %d\n", std::chrono::duration<double>(t8-t7).count()*1e3, std::chrono::duration<double>(t10-t9).count()*1e3, f2==first);
  printf("radix %.2f ms equal %d  starts2 %.2f ms equal %d\n", std::chrono::duration<double>(t5-t4).count()*1e3, vc2==vc, std::chrono::duration<double>(t6-t5).count()*1e3, st2==st);
  auto ms=[](auto a,auto b){return std::chrono::duration<double>(b-a).count()*1e3;};
  printf("distinct %zu  count %.2f ms  sort %.2f ms  starts %.2f ms\n", first.size(), ms(t0,t1), ms(t1,t2), ms(t2,t3));
  }
}

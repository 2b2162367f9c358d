#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <fcntl.h>
#include <unistd.h>
#include <sys/stat.h>
#include <thread>
using clk = std::chrono::steady_clock;
static double ms(clk::time_point a, clk::time_point b){return std::chrono::duration<double,std::milli>(b-a).count();}
int main(int argc, char** argv){
  for(int r=0;r<3;++r){
  auto t0=clk::now();
  int fd=open(argv[1],O_RDONLY); struct stat st; fstat(fd,&st);
  std::string out((size_t)st.st_size,'\0');
  auto t1=clk::now();
  size_t a=0; while(a<out.size()){ssize_t k=pread(fd,&out[a],out.size()-a,a); if(k<=0)break; a+=k;}
  close(fd);
  auto t2=clk::now();
  std::vector<uint32_t> s; s.reserve(1100000); std::vector<uint32_t> t; t.reserve(1100000);
  const char* p=strchr(out.data(),'\n')+1; const char* e=out.data()+out.size();
  while(p<e){ uint32_t x=0,y=0; while(*p>='0'&&*p<='9') x=x*10+(*p++-'0'); ++p; while(*p>='0'&&*p<='9') y=y*10+(*p++-'0'); ++p; s.push_back(x); t.push_back(y);}  
  auto t3=clk::now();
  std::printf("alloc %.2f read %.2f parse %.2f (%zu)\n", ms(t0,t1), ms(t1,t2), ms(t2,t3), s.size());
  std::vector<std::thread> th; auto t4=clk::now(); for(int i=0;i<16;++i) th.emplace_back([]{}); for(auto&x:th) x.join(); auto t5=clk::now();
  std::printf("16 thread spawn+join %.2f ms\n", ms(t4,t5));
  }
}

// Probe: can two processes on the same GPU form an RCCL communicator and exchange a buffer?
// usage: probe <rank> <nranks> <idfile>   (rank 0 writes the unique id, rank 1 reads it)
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <thread>
#include <chrono>
int main(int argc, char **argv) {
  int rank = atoi(argv[1]), n = atoi(argv[2]);
  const char *idf = argv[3];
  ncclUniqueId id;
  if (rank == 0) {
    ncclGetUniqueId(&id);
    std::ofstream f(std::string(idf) + ".tmp", std::ios::binary);
    f.write((char *)&id, sizeof(id));
    f.close();
    std::rename((std::string(idf) + ".tmp").c_str(), idf);
  } else {
    for (int t = 0; t < 300; t++) {
      std::ifstream f(idf, std::ios::binary);
      if (f.good()) { f.read((char *)&id, sizeof(id)); if (f.gcount() == sizeof(id)) break; }
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
    }
  }
  hipSetDevice(0);
  ncclComm_t comm;
  ncclResult_t r = ncclCommInitRank(&comm, n, id, rank);
  printf("rank %d init: %s\n", rank, ncclGetErrorString(r));
  if (r != ncclSuccess) return 1;
  double *buf, *rbuf;
  hipMalloc(&buf, 1024 * 8);
  hipMalloc(&rbuf, 1024 * 8);
  double h[1024];
  for (int i = 0; i < 1024; i++) h[i] = rank * 1000 + i;
  hipMemcpy(buf, h, sizeof(h), hipMemcpyHostToDevice);
  hipStream_t s;
  hipStreamCreate(&s);
  int peer = 1 - rank;
  auto t0 = std::chrono::steady_clock::now();
  for (int it = 0; it < 100; it++) {
    ncclGroupStart();
    ncclSend(buf, 1024, ncclDouble, peer, comm, s);
    ncclRecv(rbuf, 1024, ncclDouble, peer, comm, s);
    ncclGroupEnd();
  }
  hipStreamSynchronize(s);
  auto t1 = std::chrono::steady_clock::now();
  hipMemcpy(h, rbuf, sizeof(h), hipMemcpyDeviceToHost);
  printf("rank %d got %g %g, %.2f us per exchange\n", rank, h[0], h[1023],
         std::chrono::duration<double, std::micro>(t1 - t0).count() / 100);
  ncclCommDestroy(comm);
  return 0;
}

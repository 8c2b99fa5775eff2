// Hardware probe: dumps raw amd-smi values and per-call latency for every API
// the amd-smi backend uses.  Build: g++ -O2 -std=c++17 -I/opt/rocm/include
//   tools/amdsmi_probe.cpp -o build/amdsmi_probe -L/opt/rocm/lib -lamd_smi
#include <amd_smi/amdsmi.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define T(call)                                                             \
  ({                                                                        \
    double t0__ = now_us();                                                 \
    amdsmi_status_t st__ = (call);                                          \
    printf("  %-58s st=%d %8.1f us\n", #call, (int)st__, now_us() - t0__); \
    st__;                                                                   \
  })

int main(int argc, char** argv) {
  int rounds = argc > 1 ? atoi(argv[1]) : 3;
  for (int r = 0; r < rounds; ++r) {
    printf("=== round %d\n", r);
    double c0 = now_us();
    T(amdsmi_init(AMDSMI_INIT_AMD_GPUS));
    uint32_t ns = 0;
    T(amdsmi_get_socket_handles(&ns, nullptr));
    std::vector<amdsmi_socket_handle> socks(ns);
    T(amdsmi_get_socket_handles(&ns, socks.data()));
    printf("sockets=%u\n", ns);
    for (auto s : socks) {
      uint32_t np = 0;
      T(amdsmi_get_processor_handles(s, &np, nullptr));
      std::vector<amdsmi_processor_handle> procs(np);
      T(amdsmi_get_processor_handles(s, &np, procs.data()));
      printf("processors=%u\n", np);
      for (auto p : procs) {
        processor_type_t pt;
        T(amdsmi_get_processor_type(p, &pt));
        printf("type=%d\n", (int)pt);
        amdsmi_asic_info_t asic;
        memset(&asic, 0, sizeof(asic));
        T(amdsmi_get_gpu_asic_info(p, &asic));
        printf("market=%s vendor=0x%x dev=0x%lx rev=%u cus=%u tgv=%lu (0x%lx) oam=%u serial=%s\n", asic.market_name,
               asic.vendor_id, (unsigned long)asic.device_id, asic.rev_id, asic.num_of_compute_units,
               (unsigned long)asic.target_graphics_version, (unsigned long)asic.target_graphics_version, asic.oam_id,
               asic.asic_serial);
        uint64_t bdfid = 0;
        T(amdsmi_get_gpu_bdf_id(p, &bdfid));
        amdsmi_bdf_t bdf;
        T(amdsmi_get_gpu_device_bdf(p, &bdf));
        printf("bdfid=0x%lx bdf=%04lx:%02x:%02x.%x\n", (unsigned long)bdfid, (unsigned long)bdf.domain_number,
               bdf.bus_number, bdf.device_number, bdf.function_number);
        char uuid[128] = {0};
        unsigned int ulen = sizeof(uuid);
        T(amdsmi_get_gpu_device_uuid(p, &ulen, uuid));
        printf("uuid=%s\n", uuid);
        amdsmi_kfd_info_t kfd;
        T(amdsmi_get_gpu_kfd_info(p, &kfd));
        printf("kfd_id=%lu node=%u part=%u\n", (unsigned long)kfd.kfd_id, kfd.node_id, kfd.current_partition_id);
        uint64_t total = 0;
        T(amdsmi_get_gpu_memory_total(p, AMDSMI_MEM_TYPE_VRAM, &total));
        printf("vram_total=%lu\n", (unsigned long)total);
        amdsmi_vram_info_t vram;
        T(amdsmi_get_gpu_vram_info(p, &vram));
        printf("vram type=%d vendor=%s size_mb=%lu width=%lu\n", (int)vram.vram_type, vram.vram_vendor,
               (unsigned long)vram.vram_size, (unsigned long)vram.vram_bit_width);
        char cp[64] = {0}, mp[64] = {0};
        T(amdsmi_get_gpu_compute_partition(p, cp, sizeof(cp)));
        T(amdsmi_get_gpu_memory_partition(p, mp, sizeof(mp)));
        printf("compute_partition=%s memory_partition=%s\n", cp, mp);
        amdsmi_memory_partition_config_t mcfg;
        memset(&mcfg, 0, sizeof(mcfg));
        T(amdsmi_get_gpu_memory_partition_config(p, &mcfg));
        printf("mem caps=0x%x mode=%d numa=%u\n", mcfg.partition_caps.nps_cap_mask, (int)mcfg.mp_mode,
               mcfg.num_numa_ranges);
        amdsmi_accelerator_partition_profile_t prof;
        memset(&prof, 0, sizeof(prof));
        uint32_t pids[AMDSMI_MAX_ACCELERATOR_PARTITIONS] = {0};
        T(amdsmi_get_gpu_accelerator_partition_profile(p, &prof, pids));
        printf("profile type=%d nparts=%u idx=%u nres=%u memcaps=0x%x pids=%u,%u\n", (int)prof.profile_type,
               prof.num_partitions, prof.profile_index, prof.num_resources, prof.memory_caps.nps_cap_mask, pids[0],
               pids[1]);
        amdsmi_accelerator_partition_profile_config_t pcfg;
        memset(&pcfg, 0, sizeof(pcfg));
        T(amdsmi_get_gpu_accelerator_partition_profile_config(p, &pcfg));
        printf("profile_config nprof=%u nres_types=%u\n", pcfg.num_profiles, pcfg.num_resource_profiles);
        for (uint32_t i = 0; i < pcfg.num_profiles && i < AMDSMI_MAX_ACCELERATOR_PROFILE; ++i)
          printf("  profile[%u] type=%d nparts=%u memcaps=0x%x nres=%u\n", i, (int)pcfg.profiles[i].profile_type,
                 pcfg.profiles[i].num_partitions, pcfg.profiles[i].memory_caps.nps_cap_mask,
                 pcfg.profiles[i].num_resources);
        for (uint32_t i = 0; i < pcfg.num_resource_profiles && i < AMDSMI_MAX_CP_PROFILE_RESOURCES; ++i)
          printf("  res[%u] profile_index=%u type=%d inst=%u shared=%u\n", i, pcfg.resource_profiles[i].profile_index,
                 (int)pcfg.resource_profiles[i].resource_type, pcfg.resource_profiles[i].partition_resource,
                 pcfg.resource_profiles[i].num_partitions_share_resource);
        amdsmi_xgmi_link_status_t ls;
        memset(&ls, 0, sizeof(ls));
        T(amdsmi_get_gpu_xgmi_link_status(p, &ls));
        printf("xgmi total=%u:", ls.total_links);
        for (uint32_t i = 0; i < ls.total_links && i < AMDSMI_MAX_NUM_XGMI_LINKS; ++i) printf(" %d", (int)ls.status[i]);
        printf("\n");
        amdsmi_virtualization_mode_t vm;
        T(amdsmi_get_gpu_virtualization_mode(p, &vm));
        printf("virt=%d\n", (int)vm);
        uint16_t xcd = 0;
        T(amdsmi_get_gpu_xcd_counter(p, &xcd));
        printf("xcd=%u\n", xcd);
        amdsmi_driver_info_t drv;
        memset(&drv, 0, sizeof(drv));
        T(amdsmi_get_gpu_driver_info(p, &drv));
        printf("driver name=%s version=%s date=%s\n", drv.driver_name, drv.driver_version, drv.driver_date);
        amdsmi_board_info_t board;
        memset(&board, 0, sizeof(board));
        T(amdsmi_get_gpu_board_info(p, &board));
        printf("board product=%s model=%s mfr=%s\n", board.product_name, board.model_number, board.manufacturer_name);
        amdsmi_enumeration_info_t en;
        memset(&en, 0, sizeof(en));
        T(amdsmi_get_gpu_enumeration_info(p, &en));
        printf("enum drm_render=%u drm_card=%u hsa=%u hip=%u hip_uuid=%s\n", en.drm_render, en.drm_card, en.hsa_id,
               en.hip_id, en.hip_uuid);
      }
    }
    amdsmi_version_t v;
    T(amdsmi_get_lib_version(&v));
    printf("lib %u.%u.%u %s\n", v.major, v.minor, v.release, v.build ? v.build : "");
    T(amdsmi_shut_down());
    printf("cycle total %.1f us\n", now_us() - c0);
  }
  return 0;
}

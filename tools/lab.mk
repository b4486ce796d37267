# In-process A/B builds of kernel variants (tools only, never shipped):
# libsdsp_lab.so = the product objects with kern_fir_ols_os.o, kern_chan1024.o, kern_iir_wscan.o
# rebuilt under -DSDSP_OLS_LAB -DSDSP_CHAN_LAB -DSDSP_IIR_LAB (extra template
# instances, ablation switches: sdsp_lab_set_ols_variant, sdsp_lab_set_chan_ablation,
# sdsp_lab_set_iir_ablation).
#   make -f tools/lab.mk -j8
HIPCC ?= /opt/rocm/bin/hipcc
CSRC = solid_dsp_amd/csrc
OBJ = solid_dsp_amd/_build/obj
HIPFLAGS = --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-result \
           -fvisibility=hidden -Iinclude -I$(CSRC)
LAB_SRC = kern_fir_ols_os kern_chan1024 kern_iir_wscan kern_pfb
OUT = tools/_build/libsdsp_lab.so
PRODUCT_OBJS = $(filter-out $(patsubst %,$(OBJ)/%.o,$(LAB_SRC)),$(wildcard $(OBJ)/*.o))

all: $(OUT)

tools/_build/lab/%.o: $(CSRC)/%.hip $(CSRC)/*.hpp include/sdsp.h tools/lab.mk
	@mkdir -p tools/_build/lab
	$(HIPCC) $(HIPFLAGS) -DSDSP_OLS_LAB -DSDSP_CHAN_LAB -DSDSP_IIR_LAB -DSDSP_PFB_LAB -c $< -o $@

# the slot kernel's queue atomic is issued by one lane and its result is needed a segment later: no
# wave-level atomic rewrite (it waits for the returned value at once)
tools/_build/lab/kern_fir_ols_os.o: HIPFLAGS += -mllvm -amdgpu-atomic-optimizer-strategy=None

tools/_build/lab/kern_iir_wscan.o: HIPFLAGS += -fno-slp-vectorize

$(OUT): $(patsubst %,tools/_build/lab/%.o,$(LAB_SRC)) $(PRODUCT_OBJS)
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@ $^

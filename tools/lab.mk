# In-process A/B builds of kernel variants (tools only, never shipped):
# libsdsp_lab.so = the product objects, with each product TU listed in LAB_MAP
# replaced by its lab TU under tools/lab/ (the lab TU compiles the product source
# unchanged and adds launchers for other compile-time variants, selected by the
# sdsp_lab_* entry points the tools/*_ab.py / *_lab.py drivers call).
#   make -f tools/lab.mk -j8
HIPCC ?= /opt/rocm/bin/hipcc
CSRC = solid_dsp_amd/csrc
OBJ = solid_dsp_amd/_build/obj
HIPFLAGS = --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-result \
           -fvisibility=hidden -Iinclude -I$(CSRC)
# lab TU : the product object it replaces
LAB_MAP = ols_lab:kern_fir_ols_os chan_lab:kern_chan1024 iir_lab:kern_iir_wscan
LAB_TUS = $(foreach m,$(LAB_MAP),$(word 1,$(subst :, ,$(m))))
REPLACED = $(foreach m,$(LAB_MAP),$(OBJ)/$(word 2,$(subst :, ,$(m))).o)
OUT = tools/_build/libsdsp_lab.so
PRODUCT_OBJS = $(filter-out $(REPLACED),$(wildcard $(OBJ)/*.o))

all: $(OUT)

tools/_build/lab/%.o: tools/lab/%.hip $(CSRC)/*.hpp include/sdsp.h tools/lab.mk
	@mkdir -p tools/_build/lab
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# each lab TU compiles its product source
$(foreach m,$(LAB_MAP),$(eval tools/_build/lab/$(word 1,$(subst :, ,$(m))).o: $(CSRC)/$(word 2,$(subst :, ,$(m))).hip))

tools/_build/lab/iir_lab.o: HIPFLAGS += -fno-slp-vectorize
tools/_build/lab/ols_lab.o: tools/lab/ols_os_lab_kernel.hip

$(OUT): $(patsubst %,tools/_build/lab/%.o,$(LAB_TUS)) $(PRODUCT_OBJS)
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@.tmp $^ && mv -f $@.tmp $@

.PHONY: all

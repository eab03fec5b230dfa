# TEST INFRASTRUCTURE ONLY: builds oracle/_ref/libdbow2_ref.so from the reference's own
# DBoW2 BowVector.cpp and FeatureVector.cpp where they lie under REF (read-only; nothing
# is copied) plus the harness oracle/ref_dbow2_capi.cpp.  DBoW2's flags
# (Thirdparty/DBoW2/CMakeLists.txt:4-5: -Wall -O3 -march=native) with -std=c++11.  g++
# contracts a*b+c into FMA for C++ even under -std=c++11 (only ISO C keeps contraction
# off by default): this build's BowVector::normalize L2 loop holds a vfmadd, and
# tests/test_vocab_ref.py shows its output differs from an unfused build (DESIGN.md
# section 2, H4).  Nothing else of the reference builds without OpenCV.
#   make -f oracle/ref_dbow2.mk REF=/root/reference
REF ?= /root/reference
HERE := $(dir $(abspath $(lastword $(MAKEFILE_LIST))))
DB := $(REF)/Thirdparty/DBoW2/DBoW2
OUT := $(HERE)_ref/libdbow2_ref.so
CXX ?= g++

all: $(OUT)

$(OUT): $(DB)/BowVector.cpp $(DB)/FeatureVector.cpp $(HERE)ref_dbow2_capi.cpp
	mkdir -p $(HERE)_ref
	$(CXX) -std=c++11 -Wall -O3 -march=native -fPIC -shared -I$(DB) -o $@ $(DB)/BowVector.cpp \
	    $(DB)/FeatureVector.cpp $(HERE)ref_dbow2_capi.cpp

clean:
	rm -f $(OUT)
.PHONY: all clean

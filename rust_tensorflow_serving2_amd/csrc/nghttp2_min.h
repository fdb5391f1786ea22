// Minimal declarations of the libnghttp2 (v1.4x) C API used by the native
// HTTP/2 front end.  The image ships libnghttp2.so.14 but no development
// headers, so the (stable, C) ABI subset is declared here.  Only frame-header
// fields are read from nghttp2_frame, so the union is declared by its common
// leading member.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <sys/types.h>

extern "C" {

typedef struct nghttp2_session nghttp2_session;
typedef struct nghttp2_session_callbacks nghttp2_session_callbacks;
typedef struct nghttp2_option nghttp2_option;

typedef struct {
  uint8_t* name;
  uint8_t* value;
  size_t namelen;
  size_t valuelen;
  uint8_t flags;
} nghttp2_nv;

typedef struct {
  int32_t settings_id;
  uint32_t value;
} nghttp2_settings_entry;

typedef struct {
  size_t length;
  int32_t stream_id;
  uint8_t type;
  uint8_t flags;
  uint8_t reserved;
} nghttp2_frame_hd;

typedef struct {
  nghttp2_frame_hd hd;   // every frame struct in the real union starts with this
} nghttp2_frame;

typedef union {
  int fd;
  void* ptr;
} nghttp2_data_source;

typedef ssize_t (*nghttp2_data_source_read_callback)(nghttp2_session* session, int32_t stream_id, uint8_t* buf,
                                                     size_t length, uint32_t* data_flags,
                                                     nghttp2_data_source* source, void* user_data);

typedef struct {
  nghttp2_data_source source;
  nghttp2_data_source_read_callback read_callback;
} nghttp2_data_provider;

typedef int (*nghttp2_on_begin_headers_callback)(nghttp2_session*, const nghttp2_frame*, void*);
typedef int (*nghttp2_on_header_callback)(nghttp2_session*, const nghttp2_frame*, const uint8_t* name, size_t namelen,
                                          const uint8_t* value, size_t valuelen, uint8_t flags, void*);
typedef int (*nghttp2_on_frame_recv_callback)(nghttp2_session*, const nghttp2_frame*, void*);
typedef int (*nghttp2_on_data_chunk_recv_callback)(nghttp2_session*, uint8_t flags, int32_t stream_id,
                                                   const uint8_t* data, size_t len, void*);
typedef int (*nghttp2_on_stream_close_callback)(nghttp2_session*, int32_t stream_id, uint32_t error_code, void*);
typedef ssize_t (*nghttp2_send_callback)(nghttp2_session*, const uint8_t* data, size_t length, int flags, void*);
typedef int (*nghttp2_send_data_callback)(nghttp2_session*, nghttp2_frame* frame, const uint8_t* framehd,
                                          size_t length, nghttp2_data_source* source, void*);
typedef ssize_t (*nghttp2_data_source_read_length_callback)(nghttp2_session*, uint8_t frame_type, int32_t stream_id,
                                                            int32_t session_remote_window_size,
                                                            int32_t stream_remote_window_size,
                                                            uint32_t remote_max_frame_size, void*);

int nghttp2_session_callbacks_new(nghttp2_session_callbacks** callbacks_ptr);
void nghttp2_session_callbacks_del(nghttp2_session_callbacks* callbacks);
void nghttp2_session_callbacks_set_on_begin_headers_callback(nghttp2_session_callbacks*, nghttp2_on_begin_headers_callback);
void nghttp2_session_callbacks_set_on_header_callback(nghttp2_session_callbacks*, nghttp2_on_header_callback);
void nghttp2_session_callbacks_set_on_frame_recv_callback(nghttp2_session_callbacks*, nghttp2_on_frame_recv_callback);
void nghttp2_session_callbacks_set_on_data_chunk_recv_callback(nghttp2_session_callbacks*,
                                                               nghttp2_on_data_chunk_recv_callback);
void nghttp2_session_callbacks_set_on_stream_close_callback(nghttp2_session_callbacks*, nghttp2_on_stream_close_callback);
void nghttp2_session_callbacks_set_send_callback(nghttp2_session_callbacks*, nghttp2_send_callback);
void nghttp2_session_callbacks_set_send_data_callback(nghttp2_session_callbacks*, nghttp2_send_data_callback);
void nghttp2_session_callbacks_set_data_source_read_length_callback(nghttp2_session_callbacks*,
                                                                    nghttp2_data_source_read_length_callback);

int nghttp2_session_server_new(nghttp2_session** session_ptr, const nghttp2_session_callbacks* callbacks, void* user_data);
int nghttp2_session_client_new(nghttp2_session** session_ptr, const nghttp2_session_callbacks* callbacks, void* user_data);
void nghttp2_session_del(nghttp2_session* session);
ssize_t nghttp2_session_mem_recv(nghttp2_session* session, const uint8_t* in, size_t inlen);
ssize_t nghttp2_session_mem_send(nghttp2_session* session, const uint8_t** data_ptr);
int nghttp2_session_send(nghttp2_session* session);
int nghttp2_session_want_read(nghttp2_session* session);
int nghttp2_session_want_write(nghttp2_session* session);
int nghttp2_session_set_local_window_size(nghttp2_session* session, uint8_t flags, int32_t stream_id,
                                          int32_t window_size);
void* nghttp2_session_get_stream_user_data(nghttp2_session* session, int32_t stream_id);
int nghttp2_session_set_stream_user_data(nghttp2_session* session, int32_t stream_id, void* stream_user_data);
int nghttp2_session_resume_data(nghttp2_session* session, int32_t stream_id);
int nghttp2_session_terminate_session(nghttp2_session* session, uint32_t error_code);

int nghttp2_submit_settings(nghttp2_session* session, uint8_t flags, const nghttp2_settings_entry* iv, size_t niv);
int nghttp2_submit_response(nghttp2_session* session, int32_t stream_id, const nghttp2_nv* nva, size_t nvlen,
                            const nghttp2_data_provider* data_prd);
int nghttp2_submit_trailer(nghttp2_session* session, int32_t stream_id, const nghttp2_nv* nva, size_t nvlen);
int32_t nghttp2_submit_request(nghttp2_session* session, const void* pri_spec, const nghttp2_nv* nva, size_t nvlen,
                               const nghttp2_data_provider* data_prd, void* stream_user_data);
int nghttp2_submit_rst_stream(nghttp2_session* session, uint8_t flags, int32_t stream_id, uint32_t error_code);
const char* nghttp2_strerror(int lib_error_code);

}  // extern "C"

// constants (nghttp2.h)
enum : uint8_t {
  NGHTTP2_DATA = 0, NGHTTP2_HEADERS = 1, NGHTTP2_RST_STREAM = 3, NGHTTP2_SETTINGS = 4,
  NGHTTP2_GOAWAY = 7, NGHTTP2_WINDOW_UPDATE = 8,
};
enum : uint8_t { NGHTTP2_FLAG_NONE = 0, NGHTTP2_FLAG_END_STREAM = 0x01, NGHTTP2_FLAG_END_HEADERS = 0x04 };
enum : int32_t {
  NGHTTP2_SETTINGS_HEADER_TABLE_SIZE = 1, NGHTTP2_SETTINGS_ENABLE_PUSH = 2,
  NGHTTP2_SETTINGS_MAX_CONCURRENT_STREAMS = 3, NGHTTP2_SETTINGS_INITIAL_WINDOW_SIZE = 4,
  NGHTTP2_SETTINGS_MAX_FRAME_SIZE = 5, NGHTTP2_SETTINGS_MAX_HEADER_LIST_SIZE = 6,
};
enum : uint32_t { NGHTTP2_DATA_FLAG_EOF = 0x01, NGHTTP2_DATA_FLAG_NO_END_STREAM = 0x02,
                  NGHTTP2_DATA_FLAG_NO_COPY = 0x04 };
enum : uint8_t { NGHTTP2_NV_FLAG_NONE = 0, NGHTTP2_NV_FLAG_NO_COPY_NAME = 0x02, NGHTTP2_NV_FLAG_NO_COPY_VALUE = 0x04 };
enum : int { NGHTTP2_ERR_WOULDBLOCK = -504, NGHTTP2_ERR_DEFERRED = -508, NGHTTP2_ERR_CALLBACK_FAILURE = -902,
             NGHTTP2_ERR_TEMPORAL_CALLBACK_FAILURE = -521 };
enum : uint32_t { NGHTTP2_NO_ERROR = 0, NGHTTP2_INTERNAL_ERROR = 2, NGHTTP2_CANCEL = 8 };

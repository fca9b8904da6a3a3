"""NRMS hyper-parameters, field-for-field with the reference's config classes
(src/config.py:10-45) so a reference config object can be passed unchanged.
The NRMS path and the preprocessing (preprocess.py) read these fields, plus this build's own knobs
(prefixed ``hip_``)."""


class BaseConfig:
    num_epochs = 2
    num_batches_show_loss = 100
    num_batches_validate = 1000
    batch_size = 128
    learning_rate = 0.0001
    num_workers = 4
    num_clicked_news_a_user = 50
    num_words_title = 20
    num_words_abstract = 50
    word_freq_threshold = 1
    entity_freq_threshold = 2
    entity_confidence_threshold = 0.5
    negative_sampling_ratio = 2
    dropout_probability = 0.2
    num_words = 1 + 70975
    num_categories = 1 + 274
    num_entities = 1 + 12957
    num_users = 1 + 50000
    word_embedding_dim = 300
    category_embedding_dim = 100
    entity_embedding_dim = 100
    query_vector_dim = 200


class NRMSConfig(BaseConfig):
    dataset_attributes = {"news": ["title"], "record": []}
    num_attention_heads = 15
    # --- MI355X build knobs (not in the reference) ---
    hip_proj_mode = 0            # 0 auto, 1 direct, 2 folded (include/nrms_hip.h)
    hip_cache_folded_table = True  # reuse the vocab projection across get_news_vector calls
    hip_check_ids = True         # raise IndexError on out-of-range ids, like nn.Embedding

%% partisan_config shim of the in-BEAM parity harness (loaded ahead of the
%% reference's own, src/partisan_config.erl): every simulated node runs in
%% the harness process, so its configuration and identity live in the
%% process dictionary (psim_h_node = the node whose callback is running).
%% Defaults are partisan_config:init/0's (partisan_config.erl:102-145).
-module(partisan_config).
-export([init/0, get/1, get/2, set/2, seed/0, seed/1, listen_addrs/0]).

init() -> ok.

get(Key) -> get(Key, undefined).

get(name, Default) -> node_value(name, Default);
get(listen_addrs, Default) -> node_value(listen_addrs, Default);
get(Key, Default) ->
    case get({psim_h_cfg, Key}) of
        undefined -> maps:get(Key, defaults(), Default);
        V -> V
    end.

set(Key, Value) -> put({psim_h_cfg, Key}, Value), ok.

%% partisan_config:seed/0 (partisan_config.erl:159-162): the node's Philox
%% stream from draw 0 (a restarted node is re-seeded identically)
seed() ->
    Id = get(psim_h_node),
    psim_philox:install(get(random_seed_int, 1), Id, 0).
seed(_) -> seed().

listen_addrs() -> node_value(listen_addrs, []).

node_value(Key, Default) ->
    case get(psim_h_node) of
        undefined -> Default;
        Id -> maps:get(Key, psim_harness:spec(Id))
    end.

defaults() ->
    #{arwl => 5, prwl => 30, max_active_size => 6, min_active_size => 3, max_passive_size => 30,
      random_promotion => true, passive_view_shuffle_period => 10000, tracing => false,
      broadcast => false, parallelism => 1, channels => [undefined], tag => undefined,
      reservations => [], lazy_tick_period => 1000, exchange_tick_period => 10000,
      partisan_peer_service_manager => psim_h_pt_manager, disable_fast_receive => true,
      transmission_logging_mfa => undefined, exchange_selection => optimized,
      broadcast_start_exchange_limit => 1, peer_service_manager => partisan_hyparview_peer_service_manager}.
